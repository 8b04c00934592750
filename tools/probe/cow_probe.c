// Fork / copy-on-write / exit costs of a zygote-like parent on this kernel:
// 4 KB pages vs transparent huge pages, and how the pages a child writes are
// spread over 2 MB regions (each first write into a shared huge page splits
// its PMD in the child).  Prints one JSON line per case.
//   cc -O2 -o /tmp/cow_probe tools/probe/cow_probe.c && /tmp/cow_probe [MB]
//   env: COW_POPULATE=1 (MADV_POPULATE_WRITE first), COW_SETSID=1 (child setsid)
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#ifndef MADV_COLLAPSE
#define MADV_COLLAPSE 25
#endif

static double cpu_ms(struct rusage* r) {
  return (r->ru_utime.tv_sec + r->ru_stime.tv_sec) * 1e3 + (r->ru_utime.tv_usec + r->ru_stime.tv_usec) / 1e3;
}
static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 && atoi(argv[1]) >= 4 ? atoi(argv[1]) : 64;
  const size_t size = mb << 20, huge = 2 << 20;
  const int reps = 20;
  for (int thp = 0; thp <= 1; ++thp) {
    for (int spread = 0; spread <= 2; ++spread) {
      // spread 0: 512 pages packed in one 2 MB region's worth of 4 KB pages
      // (i.e. contiguous), 1: 512 pages = 16 in each of 32 regions, 2: 512
      // pages = 1 in each of 512... (capped by the region count: 16 per region)
      char* raw = mmap(NULL, size + huge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      char* base = (char*)(((unsigned long)raw + huge - 1) & ~(huge - 1));
      madvise(base, size, thp ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
      memset(base, 1, size);
      if (thp) madvise(base, size, MADV_COLLAPSE);
      const int regions = (int)(size / huge);
      const int r32 = regions < 32 ? regions : 32;  // (>= 1 MB: 512 pages fit in 2 regions)
      double fork_ms = 0, child_ms = 0, total_ms = 0, wall = 0;
      long flt = 0;
      for (int r = 0; r < reps; ++r) {
        int pfd[2];
        pipe(pfd);
        const double t0 = now_ms();
        struct rusage a, b;
        getrusage(RUSAGE_SELF, &a);
        pid_t pid = fork();
        if (pid == 0) {
          struct rusage c0, c1;
          getrusage(RUSAGE_SELF, &c0);
          int n = 0;
          if (getenv("COW_POPULATE") && spread == 0) {
            // the same 512 pages broken by one MADV_POPULATE_WRITE (no trap per page)
            madvise(base, 512 * 4096, 23 /* MADV_POPULATE_WRITE */);
          }
          for (int i = 0; i < 512; ++i) {
            size_t off;
            if (spread == 0) off = (size_t)i * 4096;
            else if (spread == 1) off = (size_t)(i % r32) * huge + (size_t)(i / r32) * 4096;
            else off = (size_t)(i % regions) * huge + (size_t)(i / regions) * 4096;
            base[off] = 2;
            ++n;
          }
          getrusage(RUSAGE_SELF, &c1);
          // COW_SETSID=1: a session (and scheduler autogroup) of its own, as a
          // sandbox leader has -- its creation and teardown land in exit_ms
          if (getenv("COW_SETSID")) setsid();
          double v[2] = {cpu_ms(&c1) - cpu_ms(&c0), (double)(c1.ru_minflt - c0.ru_minflt)};
          write(pfd[1], v, sizeof v);
          _exit(0);
        }
        getrusage(RUSAGE_SELF, &b);
        fork_ms += cpu_ms(&b) - cpu_ms(&a);
        double v[2];
        read(pfd[0], v, sizeof v);
        struct rusage cr;
        int st;
        wait4(pid, &st, 0, &cr);
        wall += now_ms() - t0;
        child_ms += v[0];
        flt += (long)v[1];
        total_ms += cpu_ms(&cr);
        close(pfd[0]);
        close(pfd[1]);
      }
      printf("{\"thp\": %d, \"mb\": %zu, \"spread\": %d, \"fork_ms\": %.3f, \"child_write_512_ms\": %.3f, \"child_flt\": %ld, "
             "\"child_total_ms\": %.3f, \"exit_ms\": %.3f}\n",
             thp, mb, spread, fork_ms / reps, child_ms / reps, flt / reps, total_ms / reps,
             (total_ms - child_ms) / reps);
      munmap(raw, size + huge);
    }
  }
  return 0;
}
