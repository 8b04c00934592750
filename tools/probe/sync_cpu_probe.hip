// Host CPU spent waiting for the GPU, by wait method (kernel broker design
// question): hipStreamSynchronize / hipEventSynchronize under
// hipDeviceScheduleBlockingSync vs hipEventQuery polling with sleeps.  A
// kernel busy-waits ~T us on the GPU clock; we measure the waiting thread's
// CPU time (CLOCK_THREAD_CPUTIME_ID) and wall time per wait.
//   hipcc --offload-arch=gfx950 -O2 tools/probe/sync_cpu_probe.hip -o build/sync_cpu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

__global__ void spin_kernel(long long cycles) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(2);
}

static double now_us(clockid_t c) {
  timespec ts;
  clock_gettime(c, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec / 1e3;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "blocking";
  unsigned flags = !strcmp(mode, "spin") ? hipDeviceScheduleSpin : !strcmp(mode, "yield") ? hipDeviceScheduleYield
                 : !strcmp(mode, "auto") ? hipDeviceScheduleAuto : hipDeviceScheduleBlockingSync;
  hipSetDeviceFlags(flags);
  hipSetDevice(0);
  int khz = 0;
  hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev, evb;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  hipEventCreateWithFlags(&evb, hipEventDisableTiming | hipEventBlockingSync);
  spin_kernel<<<1, 64, 0, s>>>(1000);
  hipStreamSynchronize(s);
  const int us_list[] = {50, 150, 400};
  for (int us : us_list) {
    const long long cycles = (long long)us * khz / 1000;
    for (int method = 0; method < 4; ++method) {
      double cpu = 0, wall = 0;
      const int iters = 40;
      for (int i = 0; i < iters; ++i) {
        spin_kernel<<<1, 64, 0, s>>>(cycles);
        const double c0 = now_us(CLOCK_THREAD_CPUTIME_ID), w0 = now_us(CLOCK_MONOTONIC);
        if (method == 0) {
          hipStreamSynchronize(s);
        } else if (method == 1) {
          hipEventRecord(ev, s);
          hipEventSynchronize(ev);
        } else if (method == 2) {
          hipEventRecord(evb, s);
          hipEventSynchronize(evb);
        } else {
          hipEventRecord(ev, s);
          int sleep_us = 10;
          while (hipEventQuery(ev) == hipErrorNotReady) {
            usleep(sleep_us);
            if (sleep_us < 80) sleep_us *= 2;
          }
        }
        cpu += now_us(CLOCK_THREAD_CPUTIME_ID) - c0;
        wall += now_us(CLOCK_MONOTONIC) - w0;
      }
      static const char* names[] = {"stream_sync", "event_sync", "event_sync_blockingflag", "query_poll_sleep"};
      printf("{\"device_flags\": \"%s\", \"kernel_us\": %d, \"method\": \"%s\", \"cpu_us\": %.1f, \"wall_us\": %.1f}\n",
             mode, us, names[method], cpu / iters, wall / iters);
    }
  }
  return 0;
}
