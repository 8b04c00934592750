// beekern: hand-written CDNA4 (gfx950) kernels that sandboxed user code calls
// in place of numpy (SURVEY.md §2.4 north-star kernel table).
//
// Conventions
//  * wave = 64 lanes (never 32); block sizes are multiples of 64.
//  * every public entry point is `extern "C"`, takes raw device pointers and
//    a hipStream_t, never allocates or synchronises (graph-capturable, G9).
//  * memory-bound kernels move 16 B per lane per access (G13) and use a
//    grid-stride loop over a grid capped at ~8 blocks per CU (G11).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <utility>
#include <type_traits>

#define BK_API extern "C" __attribute__((visibility("default")))

namespace bk {

constexpr int kWave = 64;
constexpr int kNumCU = 256;       // MI355X
constexpr int kNumXCD = 8;        // 8 XCDs x 32 CUs, private L2 each

enum Status : int {
  kOk = 0,
  kBadArgument = 1,
  kLaunchFailed = 2,
  kOutOfMemory = 3,
  kQuotaExceeded = 4,
  kNotInitialized = 5,
};

enum DType : int { kF32 = 0, kF64 = 1, kBF16 = 2, kF16 = 3, kI32 = 4, kI64 = 5 };

inline int dtype_size(int dt) {
  switch (dt) {
    case kF32: case kI32: return 4;
    case kF64: case kI64: return 8;
    case kBF16: case kF16: return 2;
  }
  return 0;
}

// grid for a memory-bound grid-stride kernel: enough blocks to fill every CU
// many times over, never more than the work needs.  The default cap of 64
// blocks/CU comes from tools/ew_sweep.py on MI355X (1e8 f64): square
// 5.36 -> 5.59 TB/s, Philox 4.43 -> 4.98 TB/s going from 8 to 64 blocks/CU
// -- the dispatcher keeps CUs fuller than a long grid-stride loop does.
constexpr int kStreamBlocksPerCU = 64;

inline unsigned stream_grid(int64_t work_items, int block, int max_blocks_per_cu = kStreamBlocksPerCU) {
  // BK_STREAM_BLOCKS_PER_CU overrides the DEFAULT cap only (tuning sweeps,
  // tools/ew_sweep.py); callers with their own cap (reductions, whose grid
  // sizes a fixed workspace) are never changed
  if (max_blocks_per_cu == kStreamBlocksPerCU) {
    if (const char* e = getenv("BK_STREAM_BLOCKS_PER_CU")) {
      const int v = atoi(e);
      if (v > 0) max_blocks_per_cu = v;
    }
  }
  int64_t need = (work_items + block - 1) / block;
  int64_t cap = (int64_t)kNumCU * max_blocks_per_cu;
  if (need < 1) need = 1;
  return (unsigned)(need < cap ? need : cap);
}

inline int launch_status() { return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed; }

// Streaming 16-B accesses.  NT = non-temporal (nt cache policy): measured on
// MI355X for 1e8 f64 (tools/probe/reduce_probe.hip) a square-copy went
// 5.70 -> 6.31 TB/s with nt loads + stores and a square-sum 5.24 -> 6.65 TB/s
// with nt loads (plus 16 loads in flight, 32 blocks/CU).  Only arrays that do
// not fit the 256 MiB Infinity Cache take the nt path: a smaller output is
// likely re-read from the cache by the next kernel.
constexpr int64_t kStreamNtBytes = 256ll << 20;
inline bool stream_nt(int64_t bytes) { return bytes >= kStreamNtBytes; }

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

template <bool NT, typename V>
__device__ __forceinline__ V ld16(const V* p) {
  static_assert(sizeof(V) == 16, "16-byte accesses only");
  if constexpr (NT) {
    u32x4_t r = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    V v;
    __builtin_memcpy(&v, &r, 16);
    return v;
  } else {
    return *p;
  }
}

template <bool NT, typename V>
__device__ __forceinline__ void st16(V* p, const V& v) {
  static_assert(sizeof(V) == 16, "16-byte accesses only");
  if constexpr (NT) {
    u32x4_t r;
    __builtin_memcpy(&r, &v, 16);
    __builtin_nontemporal_store(r, reinterpret_cast<u32x4_t*>(p));
  } else {
    *p = v;
  }
}

// 64-lane wave reduction (DPP/ds_swizzle lowering of __shfl_xor).
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Block reduction: wave sums -> LDS -> wave 0.  Result valid in thread 0.
template <typename T, int BLOCK>
__device__ __forceinline__ T block_sum(T v) {
  static_assert(BLOCK % kWave == 0 && BLOCK <= 1024, "block must be whole waves");
  constexpr int kWaves = BLOCK / kWave;
  __shared__ T partial[kWaves];
  v = wave_sum(v);
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  if (lane == 0) partial[wid] = v;
  __syncthreads();
  T r = 0;
  if (wid == 0) {
    r = lane < kWaves ? partial[lane] : T(0);
    r = wave_sum(r);
  }
  return r;
}

__device__ __forceinline__ float bf16_bits_to_float(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// round-to-nearest-even; NaN stays NaN via the hardware cvt (MI355X microarch,
// correctness boundaries row on f32->bf16).
__device__ __forceinline__ uint16_t float_to_bf16_bits(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// f64 -> bf16 through f32 (two RNE roundings, as the host's
// astype(float32) -> bf16): the empty asm pins the f32 intermediate, which
// the compiler otherwise may fold into one f64 -> bf16 rounding (it did in
// one of two kernels: 2 of 27200 values 1 ulp apart).
__device__ __forceinline__ uint16_t double_to_bf16_bits(double d) {
  float f = (float)d;
  asm volatile("" : "+v"(f));
  return float_to_bf16_bits(f);
}

}  // namespace bk
