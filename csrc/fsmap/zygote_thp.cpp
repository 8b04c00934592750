// Early huge-page arenas for sandbox zygotes, in the preloaded shim.
//
// A zygote's private memory is what every fork copies (page tables) and every
// sandbox exit tears down, so csrc/zygote/zygote_loop.cpp puts pymalloc's
// arenas on one MADV_HUGEPAGE region and collapses the rest into 2 MB pages.
// It can only do that once Python runs the zygote module: by then interpreter
// start-up has filled ~3 arenas on 4 KB pages -- the builtins, sys, site and
// encodings objects that every sandbox touches (BEE_DEBUG_ZYGOTE_MEM,
// profiles/archive/r2_s3_zygote_mem_small_pages.log).  Loaded with LD_PRELOAD, this
// constructor runs before the interpreter initialises and installs the same
// arena allocator then, when the executor asks for it in the zygote's
// environment (BEE_ZYGOTE_THP_EARLY=1; the zygote drops the variable at once,
// so its sandboxes and their exec'd programs do nothing here).
// zygote_loop.cpp adopts the region through bee_thp_region().
#include <dlfcn.h>
#include <malloc.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

namespace {

constexpr size_t kHuge = 2u << 20;

}  // namespace

extern "C" {

// shared with csrc/zygote/zygote_loop.cpp (same layout there)
struct BeeThpRegion {
  char* base;
  size_t size, used;
  void* freed[1024];
  size_t nfreed;
  size_t arenas, fallbacks;
};

}  // extern "C"

namespace {

BeeThpRegion g_region{};

void* arena_alloc(void*, size_t n) {
  BeeThpRegion& r = g_region;
  for (size_t i = 0; i < r.nfreed; ++i)
    if (r.freed[i]) {
      void* p = r.freed[i];
      r.freed[i] = r.freed[--r.nfreed];
      r.arenas++;
      return p;
    }
  if (n <= r.size - r.used) {
    void* p = r.base + r.used;
    r.used += n;
    r.arenas++;
    return p;
  }
  r.fallbacks++;
  void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  return p == MAP_FAILED ? nullptr : p;
}

void arena_free(void*, void* p, size_t n) {
  BeeThpRegion& r = g_region;
  if ((char*)p >= r.base && (char*)p < r.base + r.size) {
    if (r.nfreed < sizeof r.freed / sizeof r.freed[0]) r.freed[r.nfreed++] = p;
    return;
  }
  munmap(p, n);
}

// CPython's PyObjectArenaAllocator
struct ArenaAllocator {
  void* ctx;
  void* (*alloc)(void*, size_t);
  void (*free)(void*, void*, size_t);
};

__attribute__((constructor)) void bee_zygote_thp_early() {
  const char* e = getenv("BEE_ZYGOTE_THP_EARLY");
  if (!e || strcmp(e, "1") != 0) return;
  // the interpreter's own entry point (not linked against: a no-op in any
  // program that is not Python)
  auto set = (void (*)(ArenaAllocator*))dlsym(RTLD_DEFAULT, "PyObject_SetArenaAllocator");
  if (!set) return;
  const size_t reserve = 1ull << 30;
  char* raw = (char*)mmap(nullptr, reserve + kHuge, PROT_READ | PROT_WRITE,
                          MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (raw == MAP_FAILED) return;
  char* base = (char*)(((uintptr_t)raw + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
  if (base > raw) munmap(raw, (size_t)(base - raw));
  const size_t tail = (size_t)(raw + reserve + kHuge - (base + reserve));
  if (tail) munmap(base + reserve, tail);
  if (madvise(base, reserve, MADV_HUGEPAGE) != 0) {
    munmap(base, reserve);
    return;
  }
  g_region.base = base;
  g_region.size = reserve;
  ArenaAllocator a{nullptr, arena_alloc, arena_free};
  set(&a);  // a plain assignment in CPython: valid before Py_Initialize
  // glibc's allocations on the heap, which thp_collapse() folds into 2 MB pages
  mallopt(M_MMAP_THRESHOLD, 64 << 20);
  mallopt(M_TOP_PAD, 2 << 20);
}

}  // namespace

extern "C" __attribute__((visibility("default"))) BeeThpRegion* bee_thp_region() {
  return g_region.base ? &g_region : nullptr;
}
