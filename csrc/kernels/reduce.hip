// Deterministic two-stage reductions: sum, fused square-sum, abs-sum, dot,
// max, min.  `numpy.sum(numpy.square(x))` of the benchmark payload
// (`examples/benchmark-numpy.py:21`) is kRedSquareSum on f64 — one HBM pass
// (800 MB read for 1e8 f64) instead of numpy's write-then-read of x².
//
// One launch: <= 32 blocks per CU, each lane streams 16-B vectors (16 in
// flight, non-temporal past the Infinity Cache), accumulates in f64,
// wave-reduces over 64 lanes (DPP) -> LDS -> one partial per block; the block
// that takes the last completion ticket folds every partial in a fixed order
// (index order, the same tree whichever block is last).  No float atomics,
// so results are bitwise reproducible run to run.  (A second single-block
// launch used to do the fold: under concurrent sandboxes it queued behind
// other tenants' GEMMs holding every CU -- 25 us mean for a 1.8 us kernel,
// profiles/archive/r2_s3_final_served_path_kernels.csv.)
#include <cstring>

#include "bk_common.hpp"
#include "bk_philox.hpp"

// The completion-ticket fold below relies on GFX9-family memory semantics:
// vmcnt counts stores and sc1 (agent-scope) accesses are coherent across
// XCDs.  gfx10+ counts stores in vscnt, so the fold could read partials that
// have not landed -- refuse to build for anything but gfx9 (gfx950 here).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "reduce.hip: the single-pass ticket fold is written for GFX9-family (gfx950) memory semantics"
#endif

namespace bk {

// kRedMaxAbsDiff: max |a - b| (two operands, like kRedDot) -- one pass where
// subtract + abs + max would be three (e.g. a row check against a reference)
enum ReduceOp : int { kRedSum = 0, kRedSquareSum, kRedAbsSum, kRedMax, kRedMin, kRedDot, kRedMaxAbsDiff, kRedCount };
template <int OP> constexpr bool kTwoOperands = OP == kRedDot || OP == kRedMaxAbsDiff;

constexpr int kRedBlock = 256;
// stage-1 grid cap, and the workspace length: 32 blocks per CU with 16 loads
// in flight per lane (tools/probe/reduce_probe.hip: 1e8 f64 square-sum
// 152 -> 120 us, 5.2 -> 6.6 TB/s, with non-temporal loads)
// (the workspace holds kRedMaxBlocks partials; the default grid is
// kRedBlocks, BK_REDUCE_BLOCKS overrides it up to the workspace for sweeps)
constexpr int kRedMaxBlocks = 32768;
// 512 blocks (2 per CU, 8 waves, 16 x 16-B loads in flight per lane):
// tools/reduce_sweep.py on MI355X, 1e8 f64 square-sum, median of 20 --
// grid-stride layout 167 / 135 / 141 / 154 / 164 / 178 us at 256 / 512 / 768 /
// 1024 / 2048 / 4096 blocks, block-contiguous 168 / 142 / 145 / 145 / 157 /
// 158; torch.sum over the same 800 MB 139 us (profiles/archive/r4_reduce_sweep*.jsonl;
// the old 8192-block grid: 175-178 us).  Round 4 (profiles/archive/r4_reduce_layout_sweep.jsonl,
// interleaved): the LDS-DMA stream below 140-145 us at its best grid (256
// blocks), the same as this kernel at 512; 4 or 8 loads in flight per lane
// instead of 16 at 512 / 1024 / 2048 blocks: 137.7 / 164-167 / 166-172 us --
// the grid (8 waves per CU), not the bytes in flight, sets the rate, and
// ~5.8 TB/s (torch.sum's too) is this read stream's ceiling on these boxes
constexpr int kRedBlocks = 512;
constexpr int kRedUnroll = 16;
// the fused RNG->reduce kernels are VALU-bound (80% of SIMD cycles issue
// VALU, profiles/archive/r4_payload_kernels_pmc.csv): 8 blocks per CU (8 waves per
// SIMD) hide more of each Philox chain's latency -- 1e8 f64 square-sum
// 91.3-91.5 us at 1024 blocks, 89.3-89.5 at 2048, 89.9-90.8 at 3072,
// 90.5-91.2 at 4096, 101.9 at 8192 (profiles/archive/r4_rand_reduce_sweep.jsonl)
constexpr int kRandRedMaxBlocks = 2048;

// lab overrides of grid targets (positive integers; anything else = default)
inline int64_t env_int(const char* name, int64_t dflt) {
  const char* e = getenv(name);
  const long long v = e ? atoll(e) : 0;
  return v > 0 ? (int64_t)v : dflt;
}

template <typename T> __device__ __forceinline__ double to_f64(T v);
template <> __device__ __forceinline__ double to_f64<double>(double v) { return v; }
template <> __device__ __forceinline__ double to_f64<float>(float v) { return (double)v; }
template <> __device__ __forceinline__ double to_f64<uint16_t>(uint16_t v) { return (double)bf16_bits_to_float(v); }

template <int OP> __device__ __forceinline__ double red_init() {
  if constexpr (OP == kRedMax) return -INFINITY;
  else if constexpr (OP == kRedMaxAbsDiff) return 0.0;
  else if constexpr (OP == kRedMin) return INFINITY;
  else return 0.0;
}
template <int OP> __device__ __forceinline__ double red_map(double a, double b) {
  if constexpr (OP == kRedSquareSum) return a * a;
  else if constexpr (OP == kRedAbsSum) return fabs(a);
  else if constexpr (OP == kRedDot) return a * b;
  else if constexpr (OP == kRedMaxAbsDiff) return fabs(a - b);
  else return a;
}
// max / min propagate NaN as numpy's max() / min() do (fmax / fmin are IEEE
// maxNum: they drop a NaN operand, so a max-abs-difference check of a result
// holding NaN would return a finite "error")
template <int OP> __device__ __forceinline__ double red_combine(double x, double y) {
  if constexpr (OP == kRedMax || OP == kRedMaxAbsDiff) return (x != x || y != y) ? __builtin_nan("") : fmax(x, y);
  else if constexpr (OP == kRedMin) return (x != x || y != y) ? __builtin_nan("") : fmin(x, y);
  else return x + y;
}

template <int OP> __device__ __forceinline__ double wave_reduce(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = red_combine<OP>(v, __shfl_xor(v, off, kWave));
  return v;
}

template <int OP> __device__ __forceinline__ double block_reduce(double v) {
  constexpr int kWaves = kRedBlock / kWave;
  __shared__ double partial[kWaves];
  v = wave_reduce<OP>(v);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) partial[wid] = v;
  __syncthreads();
  double r = red_init<OP>();
  if (wid == 0) {
    r = lane < kWaves ? partial[lane] : red_init<OP>();
    r = wave_reduce<OP>(r);
  }
  return r;
}

template <typename T> struct alignas(16) V16 { T v[16 / sizeof(T)]; };

// ---- single-launch completion ------------------------------------------------
// Every block publishes its partial, then takes a ticket; the block holding
// the last ticket folds the partials and re-arms the ticket for the next
// launch on this workspace.  Tickets start at zero (bk_reduce_workspace_init).
//
// Blocks sit on different XCDs, each with its own L2.  Partials are written
// and read with agent-scope (sc1) accesses, which are coherent across XCDs;
// a store is complete (vmcnt: GFX9 counts stores there) before its block's
// ticket.  No release/acquire fences: at agent scope those write back and
// invalidate the whole L2 (buffer_wbl2 / buffer_inv), per block -- what the
// first version of this did cost every reduction ~1 ms under concurrent
// sandboxes.
__device__ __forceinline__ void publish(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool take_last_ticket(unsigned* ticket, unsigned count) {
  __shared__ bool last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == count - 1;
  }
  __syncthreads();
  return last;
}
__device__ __forceinline__ double load_agent(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void rearm(unsigned* ticket) {
  __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the fold of `count` partials into *out by the last block
template <int OP>
__device__ __forceinline__ void finish(double v, double* partials, unsigned* ticket, double* out) {
  if (threadIdx.x == 0) publish(partials + blockIdx.x, v);
  if (!take_last_ticket(ticket, gridDim.x)) return;
  // 8 partial loads in flight per lane: they miss this XCD's L2, and one at
  // a time the fold of 8192 partials (32 per lane) was a serial chain of
  // memory latencies at the end of every reduction.  Fixed order per grid.
  constexpr int F = 8;
  const int count = (int)gridDim.x;
  double r = red_init<OP>();
  for (int i = threadIdx.x; i < count; i += F * kRedBlock) {
    double t[F];
#pragma unroll
    for (int u = 0; u < F; ++u) t[u] = i + u * kRedBlock < count ? load_agent(partials + i + u * kRedBlock) : red_init<OP>();
#pragma unroll
    for (int u = 0; u < F; ++u) r = red_combine<OP>(r, t[u]);
  }
  r = block_reduce<OP>(r);
  if (threadIdx.x == 0) {
    *out = r;
    rearm(ticket);
  }
}

template <typename T, int OP, bool NT, int U = kRedUnroll>  // U: 16-B loads in flight per lane
__global__ __launch_bounds__(kRedBlock) void reduce_1pass(const T* __restrict__ a, const T* __restrict__ b, int64_t n,
                                                         double* __restrict__ partials, unsigned* __restrict__ ticket,
                                                         double* __restrict__ out) {
  using V = V16<T>;
  constexpr int N = 16 / sizeof(T);
  const int64_t nvec = n / N;
  const int64_t stride = (int64_t)gridDim.x * kRedBlock;
  const int64_t tid = (int64_t)blockIdx.x * kRedBlock + threadIdx.x;
  double acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = red_init<OP>();

  int64_t i = tid;
  for (; i + (U - 1) * stride < nvec; i += U * stride) {
    V va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = ld16<NT>(reinterpret_cast<const V*>(a) + i + u * stride);
      if constexpr (kTwoOperands<OP>) vb[u] = ld16<NT>(reinterpret_cast<const V*>(b) + i + u * stride);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const double bj = kTwoOperands<OP> ? to_f64<T>(vb[u].v[j]) : 0.0;
        acc[u] = red_combine<OP>(acc[u], red_map<OP>(to_f64<T>(va[u].v[j]), bj));
      }
  }
  // the rest in groups of 4 loads in flight: at 1e8 f64 on the capped grid a
  // lane has ~24 vectors, 16 + 8 -- one at a time, the last 8 cost as much
  // as the first 16
  constexpr int U2 = 4;
  for (; i + (U2 - 1) * stride < nvec; i += U2 * stride) {
    V va[U2], vb[U2];
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      va[u] = ld16<NT>(reinterpret_cast<const V*>(a) + i + u * stride);
      if constexpr (kTwoOperands<OP>) vb[u] = ld16<NT>(reinterpret_cast<const V*>(b) + i + u * stride);
    }
#pragma unroll
    for (int u = 0; u < U2; ++u)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const double bj = kTwoOperands<OP> ? to_f64<T>(vb[u].v[j]) : 0.0;
        acc[u] = red_combine<OP>(acc[u], red_map<OP>(to_f64<T>(va[u].v[j]), bj));
      }
  }
  for (; i < nvec; i += stride) {
    V va = reinterpret_cast<const V*>(a)[i];
    V vb;
    if constexpr (kTwoOperands<OP>) vb = reinterpret_cast<const V*>(b)[i];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double bj = kTwoOperands<OP> ? to_f64<T>(vb.v[j]) : 0.0;
      acc[0] = red_combine<OP>(acc[0], red_map<OP>(to_f64<T>(va.v[j]), bj));
    }
  }
  for (int64_t k = nvec * N + tid; k < n; k += stride) {
    const double bk_ = kTwoOperands<OP> ? to_f64<T>(b[k]) : 0.0;
    acc[0] = red_combine<OP>(acc[0], red_map<OP>(to_f64<T>(a[k]), bk_));
  }
  double v = acc[0];
#pragma unroll
  for (int u = 1; u < U; ++u) v = red_combine<OP>(v, acc[u]);
  finish<OP>(block_reduce<OP>(v), partials, ticket, out);
}

// Block-contiguous layout: block b owns one contiguous run of the array and
// its lanes walk it 16 vectors (64 KiB per 256-lane block) at a time, so a
// block's 16 loads in flight are consecutive 4 KiB stripes.  The grid-stride
// layout above puts a lane's 16 loads gridDim x 4 KiB apart (32 MiB at 8192
// blocks) -- every wave of the chip then hits the same few power-of-two
// address strides at once (a channel-camping pattern); here the concurrent
// reads are spread over the whole array.  Opt-in (BK_REDUCE_LAYOUT=chunk):
// at the 512-block grid the grid-stride kernel measured faster
// (tools/reduce_sweep.py, kRedBlocks).
template <typename T, int OP, bool NT>
__global__ __launch_bounds__(kRedBlock) void reduce_chunked(const T* __restrict__ a, const T* __restrict__ b,
                                                           int64_t n, double* __restrict__ partials,
                                                           unsigned* __restrict__ ticket, double* __restrict__ out) {
  using V = V16<T>;
  constexpr int N = 16 / sizeof(T);
  constexpr int U = kRedUnroll;
  const int64_t nvec = n / N;
  // runs of whole 256-vector stripes, the last block takes what is left
  const int64_t stripes = (nvec + kRedBlock - 1) / kRedBlock;
  const int64_t per = (stripes + gridDim.x - 1) / gridDim.x;
  const int64_t v0 = (int64_t)blockIdx.x * per * kRedBlock;
  const int64_t v1 = v0 + per * kRedBlock < nvec ? v0 + per * kRedBlock : nvec;
  double acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = red_init<OP>();
  int64_t i = v0 + threadIdx.x;
  for (; i + (int64_t)(U - 1) * kRedBlock < v1; i += (int64_t)U * kRedBlock) {
    V va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = ld16<NT>(reinterpret_cast<const V*>(a) + i + u * kRedBlock);
      if constexpr (kTwoOperands<OP>) vb[u] = ld16<NT>(reinterpret_cast<const V*>(b) + i + u * kRedBlock);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const double bj = kTwoOperands<OP> ? to_f64<T>(vb[u].v[j]) : 0.0;
        acc[u] = red_combine<OP>(acc[u], red_map<OP>(to_f64<T>(va[u].v[j]), bj));
      }
  }
  for (; i < v1; i += kRedBlock) {
    V va = ld16<NT>(reinterpret_cast<const V*>(a) + i);
    V vb;
    if constexpr (kTwoOperands<OP>) vb = ld16<NT>(reinterpret_cast<const V*>(b) + i);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double bj = kTwoOperands<OP> ? to_f64<T>(vb.v[j]) : 0.0;
      acc[0] = red_combine<OP>(acc[0], red_map<OP>(to_f64<T>(va.v[j]), bj));
    }
  }
  // the scalar tail (n % N elements) in the last block
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t k = nvec * N + threadIdx.x; k < n; k += kRedBlock) {
      const double bk_ = kTwoOperands<OP> ? to_f64<T>(b[k]) : 0.0;
      acc[0] = red_combine<OP>(acc[0], red_map<OP>(to_f64<T>(a[k]), bk_));
    }
  double v = acc[0];
#pragma unroll
  for (int u = 1; u < U; ++u) v = red_combine<OP>(v, acc[u]);
  finish<OP>(block_reduce<OP>(v), partials, ticket, out);
}

// LDS-DMA stream: each wave walks one contiguous run of 1-KiB pieces (a
// wave's 64 lanes x 16 B) through a private ring of kDmaSlots pieces in LDS,
// filled by `global_load_lds_dwordx4` (non-temporal for arrays past the
// Infinity Cache), kDmaSlots pieces in flight; it reads its own lanes' 16 B
// back with ds_read_b128 once the covering `s_waitcnt vmcnt` says they
// landed.  MI355X_MICROARCH.md measures an LDS-DMA stream at 6.4 TB/s
// (6.5-6.8 nt) against ~6.3 for register-staged copies; the register-load
// kernels above reach 5.7 TB/s on this reduction (torch.sum 5.8,
// profiles/archive/r4_reduce_sweep3.jsonl).  Measured, it does not beat them: 144-145
// us per-wave contiguous, 139-141 us with grid-strided pieces (STRIDED), both
// at 256 blocks; slower at 512+ (profiles/archive/r4_reduce_layout_sweep.jsonl).  A lab
// layout (BK_REDUCE_LAYOUT=ldsdma / ldsdma_stride), exact against fp64 numpy
// (tools/probe/reduce_layout_check.py).  Only the issuing wave reads a slot, so
// no barrier orders the ring: vmcnt before the read, lgkmcnt(0) before the
// slot's next fill.  The DMA is inline asm so the compiler neither tracks it
// nor inserts its own vmcnt(0) ahead of every LDS read (the GEMM's reason,
// gemm256w4_impl.hpp glds_raw).  Single-operand ops (the payload's
// square-sum); the loads use 64-bit addresses (no 4 GiB buffer limit).
constexpr int kDmaSlots = 16;  // pieces in flight per wave (16 KiB of LDS per wave, 64 KiB per block)
constexpr int kDmaGroup = 4;   // pieces retired per wait
typedef __attribute__((address_space(3))) void* red_lds_ptr;

template <bool NT>
__device__ __forceinline__ void dma_piece(const void* src, unsigned lds_addr) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_addr);
  // s_nop 0: one wait state between the M0 write and the LDS-DMA load
  if constexpr (NT)
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m0), "v"(src) : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(src) : "memory", "m0");
}

template <typename T, int OP, bool NT, bool STRIDED>
__global__ __launch_bounds__(kRedBlock) void reduce_ldsdma(const T* __restrict__ a, int64_t n,
                                                          double* __restrict__ partials, unsigned* __restrict__ ticket,
                                                          double* __restrict__ out) {
  static_assert(!kTwoOperands<OP>, "single-operand reductions");
  constexpr int N = 16 / sizeof(T);
  constexpr int S = kDmaSlots, G = kDmaGroup;
  __shared__ __attribute__((aligned(1024))) char ring[kRedBlock / kWave][S * 1024];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t pieces = n / (N * kWave);  // whole 1-KiB pieces
  const int64_t waves = (int64_t)gridDim.x * (kRedBlock / kWave);
  const int64_t per = (pieces + waves - 1) / waves;
  const int64_t w = (int64_t)blockIdx.x * (kRedBlock / kWave) + wid;
  // STRIDED: wave w takes pieces w, w + waves, ... (the whole chip sweeps one
  // contiguous front, as the grid-stride kernel does); else one contiguous run
  const int64_t p0 = STRIDED ? w : (w * per < pieces ? w * per : pieces);
  const int64_t np = STRIDED ? (w < pieces ? (pieces - w + waves - 1) / waves : 0)
                             : (p0 + per < pieces ? p0 + per : pieces) - p0;
  const int64_t step = STRIDED ? waves * 1024 : 1024;  // bytes from one of this wave's pieces to the next
  const char* src = reinterpret_cast<const char*>(a) + p0 * 1024 + lane * 16;
  const unsigned base = (unsigned)(unsigned long long)(red_lds_ptr)(&ring[wid][0]);
  const char* mine = &ring[wid][lane * 16];
  double acc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g] = red_init<OP>();
  auto take = [&](double& r, int slot) {
    const V16<T> v = *reinterpret_cast<const V16<T>*>(mine + slot * 1024);
#pragma unroll
    for (int q = 0; q < N; ++q) r = red_combine<OP>(r, red_map<OP>(to_f64<T>(v.v[q]), 0.0));
  };
  const int64_t first = np < S ? np : S;
  for (int64_t j = 0; j < first; ++j) dma_piece<NT>(src + j * step, base + (unsigned)j * 1024);
  int64_t j = 0;
  // steady state: exactly S pieces in flight before each wait
  for (; j + S + G <= np; j += G) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S - G) : "memory");
#pragma unroll
    for (int g = 0; g < G; ++g) take(acc[g], (int)((j + g) % S));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slots' reads are done before their refill
#pragma unroll
    for (int g = 0; g < G; ++g)
      dma_piece<NT>(src + (j + S + g) * step, base + (unsigned)((j + g) % S) * 1024);
  }
  // the rest: everything issued so far lands, then the pieces never issued
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int64_t issued = j + S < np ? j + S : np;
  for (int64_t k = j; k < issued; ++k) take(acc[0], (int)(k % S));
  for (int64_t k = issued; k < np; ++k) {
    const V16<T> v = ld16<NT>(reinterpret_cast<const V16<T>*>(src + k * step));
#pragma unroll
    for (int q = 0; q < N; ++q) acc[0] = red_combine<OP>(acc[0], red_map<OP>(to_f64<T>(v.v[q]), 0.0));
  }
  // elements past the last whole piece: the grid's last block
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t k = pieces * N * kWave + threadIdx.x; k < n; k += kRedBlock)
      acc[0] = red_combine<OP>(acc[0], red_map<OP>(to_f64<T>(a[k]), 0.0));
  double v = acc[0];
#pragma unroll
  for (int g = 1; g < G; ++g) v = red_combine<OP>(v, acc[g]);
  finish<OP>(block_reduce<OP>(v), partials, ticket, out);
}

// ---- fused RNG -> reduce -------------------------------------------------------
// sum / square-sum over a uniform Philox stream WITHOUT materialising it:
// element i takes exactly the value philox_uniform_{f64,f32} would store
// (same counter, tag and construction, bk_philox.hpp), so the result equals
// the reduction of the materialised draw up to summation order.  This is what
// `bk.sum(bk.square(bk.random.rand(n)))` lowers to while the draw is still
// lazy (ops/array.py): compute-bound (Philox) instead of 2 x n x 8 bytes of
// HBM traffic.  Two counters per iteration keep two independent Philox
// chains in flight per lane.
template <int OP>
__device__ __forceinline__ double rr_map(double v) {
  return OP == kRedSquareSum ? v * v : v;
}

template <int OP>
__global__ __launch_bounds__(kRedBlock) void rand_reduce_f64(int64_t n, uint32_t k0, uint32_t k1, uint64_t offset,
                                                             double lo, double span, double* __restrict__ partials,
                                                             unsigned* __restrict__ ticket, double* __restrict__ out) {
  const int64_t pairs = (n + 1) / 2, full = n / 2;  // `full`: pairs whose both values are in range
  const int64_t stride = (int64_t)gridDim.x * kRedBlock;
  // lo + span * (X * 2^-53) as ONE fma of the 53-bit integer X: span * 2^-53
  // is exact, so X * s53 is the same real number as span * u and the fused
  // result has the same bits as the materialised draw's fma(span, u, lo) --
  // one f64 multiply per value fewer in a VALU-bound loop
  const double s53 = span * (1.0 / 9007199254740992.0);
  auto draw = [&](uint32_t a, uint32_t b) { return fma(u53_int(a, b), s53, lo); };
  double acc0 = 0.0, acc1 = 0.0;
  int64_t p = (int64_t)blockIdx.x * kRedBlock + threadIdx.x;
  for (; p + stride < full; p += 2 * stride) {
    const uint64_t c0 = offset + (uint64_t)p, c1 = c0 + (uint64_t)stride;
    const uint4 r0 = Philox::run(make_uint4((uint32_t)c0, (uint32_t)(c0 >> 32), kTagUniformF64, 0u), k0, k1);
    const uint4 r1 = Philox::run(make_uint4((uint32_t)c1, (uint32_t)(c1 >> 32), kTagUniformF64, 0u), k0, k1);
    acc0 += rr_map<OP>(draw(r0.x, r0.y)) + rr_map<OP>(draw(r0.z, r0.w));
    acc1 += rr_map<OP>(draw(r1.x, r1.y)) + rr_map<OP>(draw(r1.z, r1.w));
  }
  for (; p < pairs; p += stride) {
    const uint64_t c0 = offset + (uint64_t)p;
    const uint4 r0 = Philox::run(make_uint4((uint32_t)c0, (uint32_t)(c0 >> 32), kTagUniformF64, 0u), k0, k1);
    acc0 += rr_map<OP>(draw(r0.x, r0.y));
    if (2 * p + 1 < n) acc0 += rr_map<OP>(draw(r0.z, r0.w));
  }
  finish<OP>(block_reduce<OP>(acc0 + acc1), partials, ticket, out);
}

template <int OP>
__global__ __launch_bounds__(kRedBlock) void rand_reduce_f32(int64_t n, uint32_t k0, uint32_t k1, uint64_t offset,
                                                             float lo, float span, double* __restrict__ partials,
                                                             unsigned* __restrict__ ticket, double* __restrict__ out) {
  const int64_t quads = (n + 3) / 4;
  const int64_t stride = (int64_t)gridDim.x * kRedBlock;
  double acc = 0.0;
  for (int64_t q = (int64_t)blockIdx.x * kRedBlock + threadIdx.x; q < quads; q += stride) {
    const uint64_t c = offset + (uint64_t)q;
    const uint4 r = Philox::run(make_uint4((uint32_t)c, (uint32_t)(c >> 32), kTagUniformF32, 0u), k0, k1);
    const float v[4] = {lo + span * u24(r.x), lo + span * u24(r.y), lo + span * u24(r.z), lo + span * u24(r.w)};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4 * q + j < n) acc += rr_map<OP>((double)v[j]);
  }
  finish<OP>(block_reduce<OP>(acc), partials, ticket, out);
}

template <typename T, int OP>
int launch_reduce(const void* a, const void* b, int64_t n, double* workspace, double* out, hipStream_t s) {
  constexpr int N = 16 / sizeof(T);
  int64_t lanes_needed = (n / N + 3) / 4;  // 4 vectors per lane minimum before adding blocks
  static const int64_t red_blocks = env_int("BK_REDUCE_BLOCKS", kRedBlocks) <= kRedMaxBlocks
                                        ? env_int("BK_REDUCE_BLOCKS", kRedBlocks)
                                        : kRedBlocks;
  unsigned g = stream_grid(lanes_needed > 0 ? lanes_needed : 1, kRedBlock, (int)(red_blocks / kNumCU));
  if (g > (unsigned)red_blocks) g = (unsigned)red_blocks;  // the workspace holds kRedMaxBlocks partials
  unsigned* ticket = reinterpret_cast<unsigned*>(workspace + kRedMaxBlocks);
  static const bool chunked = getenv("BK_REDUCE_LAYOUT") && !strcmp(getenv("BK_REDUCE_LAYOUT"), "chunk");
  static const bool ldsdma = getenv("BK_REDUCE_LAYOUT") && !strcmp(getenv("BK_REDUCE_LAYOUT"), "ldsdma");
  static const bool ldsdma_s = getenv("BK_REDUCE_LAYOUT") && !strcmp(getenv("BK_REDUCE_LAYOUT"), "ldsdma_stride");
  const bool nt = stream_nt(n * (int64_t)sizeof(T) * (kTwoOperands<OP> ? 2 : 1));
  if constexpr (!kTwoOperands<OP>) {
    if (ldsdma || ldsdma_s) {
      if (ldsdma_s) {
        if (nt) reduce_ldsdma<T, OP, true, true><<<g, kRedBlock, 0, s>>>((const T*)a, n, workspace, ticket, out);
        else reduce_ldsdma<T, OP, false, true><<<g, kRedBlock, 0, s>>>((const T*)a, n, workspace, ticket, out);
      } else if (nt) {
        reduce_ldsdma<T, OP, true, false><<<g, kRedBlock, 0, s>>>((const T*)a, n, workspace, ticket, out);
      } else {
        reduce_ldsdma<T, OP, false, false><<<g, kRedBlock, 0, s>>>((const T*)a, n, workspace, ticket, out);
      }
      return launch_status();
    }
  }
  if (chunked) {
    if (nt) reduce_chunked<T, OP, true><<<g, kRedBlock, 0, s>>>((const T*)a, (const T*)b, n, workspace, ticket, out);
    else reduce_chunked<T, OP, false><<<g, kRedBlock, 0, s>>>((const T*)a, (const T*)b, n, workspace, ticket, out);
  } else if (nt) {
    // lab: BK_REDUCE_UNROLL=4/8 -- fewer loads in flight per lane, for grids with more waves
    static const int unroll = (int)env_int("BK_REDUCE_UNROLL", kRedUnroll);
    if (unroll == 4)
      reduce_1pass<T, OP, true, 4><<<g, kRedBlock, 0, s>>>((const T*)a, (const T*)b, n, workspace, ticket, out);
    else if (unroll == 8)
      reduce_1pass<T, OP, true, 8><<<g, kRedBlock, 0, s>>>((const T*)a, (const T*)b, n, workspace, ticket, out);
    else
      reduce_1pass<T, OP, true><<<g, kRedBlock, 0, s>>>((const T*)a, (const T*)b, n, workspace, ticket, out);
  } else {
    reduce_1pass<T, OP, false><<<g, kRedBlock, 0, s>>>((const T*)a, (const T*)b, n, workspace, ticket, out);
  }
  return launch_status();
}

template <typename T, int... OPS>
int dispatch_reduce(int op, const void* a, const void* b, int64_t n, double* ws, double* out, hipStream_t s,
                    std::integer_sequence<int, OPS...>) {
  int rc = kBadArgument;
  ((op == OPS ? (rc = launch_reduce<T, OPS>(a, b, n, ws, out, s), 0) : 0), ...);
  return rc;
}

// ---- axis reductions of a 2-D row-major matrix (numpy sum/mean(axis=)) -------
// axis 0 (per column): a block of 256 threads owns 256 columns of one row
// chunk -- each thread walks its column down the chunk, so every wave-row
// load is 64 consecutive elements; the chunk partials (f64) land in the
// workspace and the last chunk block of each column block (completion
// tickets, as above) folds them in chunk order (deterministic) -- one launch.
// axis 1 (per row): one wave per row, lanes stride the row, DPP wave sum.
constexpr int64_t kAxisWsDoubles = 1 << 18;  // 2 MiB: chunks x columns partials
constexpr int64_t kAxisTickets = 4096;       // one per column block (<= 2048 at 262144 columns)

// out[col] = scale * the chunk partials of `col` folded in a fixed order: four
// chains (chunks c, c+4, c+8, c+12) so a thread's loads are in flight together
__device__ __forceinline__ double fold_chunks(const double* part, int chunks, int64_t cols, int64_t col) {
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  int c = 0;
  for (; c + 15 < chunks; c += 16)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] += load_agent(part + (int64_t)(c + 4 * j + q) * cols + col);
  for (; c < chunks; ++c) a[c & 3] += load_agent(part + (int64_t)c * cols + col);
  return (a[0] + a[1]) + (a[2] + a[3]);
}

template <typename T, typename TO>
__global__ __launch_bounds__(256) void colsum_1pass(const T* __restrict__ x, int64_t rows, int64_t cols, int64_t ld,
                                                    int64_t rows_per_chunk, double* __restrict__ part,
                                                    unsigned* __restrict__ tickets, TO* __restrict__ out, double scale) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col < cols) {
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
    const int64_t r1 = r0 + rows_per_chunk < rows ? r0 + rows_per_chunk : rows;
    double a0 = 0.0, a1 = 0.0;
    int64_t r = r0;
    for (; r + 1 < r1; r += 2) {
      a0 += to_f64<T>(x[r * ld + col]);
      a1 += to_f64<T>(x[(r + 1) * ld + col]);
    }
    if (r < r1) a0 += to_f64<T>(x[r * ld + col]);
    publish(part + (int64_t)blockIdx.y * cols + col, a0 + a1);
  }
  if (!take_last_ticket(tickets + blockIdx.x, gridDim.y)) return;
  if (col < cols) out[col] = (TO)(fold_chunks(part, (int)gridDim.y, cols, col) * scale);
  if (threadIdx.x == 0) rearm(tickets + blockIdx.x);
}

// Column sums, 16-B vectors: a block of 16 waves owns a 16*V-column strip
// (bf16: 128 columns) of one row chunk.  A wave covers 4 rows x the strip
// per step (16 lanes per row: 256-B row segments), the block 64 rows, and
// every lane has up to four steps' loads in flight.  Lanes 16 apart hold the
// same columns: the wave folds them with cross-lane moves (fixed order), the
// block folds its 16 waves through 16 KiB of LDS, and one f64 partial per
// column and chunk goes to the workspace.  The last block of each strip
// (completion ticket) folds the strip's chunk partials in chunk order.  Narrow
// strips keep the chunk count low (4096^2: 32 strips x 32 chunks) -- the
// 512-column version spent most of its 13.6-15.4 us folding 64 chunks.
constexpr int kColWaves = 16;

template <typename T, typename TO>
__global__ __launch_bounds__(kColWaves * 64) void colsum_tile_v(const T* __restrict__ x, int64_t rows, int64_t cols,
                                                              int64_t ld, int64_t rows_per_chunk,
                                                              double* __restrict__ part, unsigned* __restrict__ tickets,
                                                              TO* __restrict__ out, double scale) {
  constexpr int V = 16 / sizeof(T);
  constexpr int W = 16 * V;  // strip width (columns)
  __shared__ double sacc[kColWaves][W];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cl = lane & 15, rl = lane >> 4;  // column lane, row lane
  const int64_t col0 = (int64_t)blockIdx.x * W + cl * V;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = r0 + rows_per_chunk < rows ? r0 + rows_per_chunk : rows;
  constexpr int kStep = kColWaves * 4;  // rows per block step
  double acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.0;
  if (col0 < cols) {
    int64_t r = r0 + wave * 4 + rl;
    for (; r + 3 * kStep < r1; r += 4 * kStep) {
      V16<T> v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const V16<T>*>(x + (r + q * kStep) * ld + col0);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += to_f64<T>(v[q].v[j]);
    }
    for (; r < r1; r += kStep) {
      const V16<T> v = *reinterpret_cast<const V16<T>*>(x + r * ld + col0);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += to_f64<T>(v.v[j]);
    }
  }
  // row lanes 0..3 of each column lane: (0 + 1) + (2 + 3), same in every lane
#pragma unroll
  for (int j = 0; j < V; ++j) {
    acc[j] += __shfl_xor(acc[j], 16, 64);
    acc[j] += __shfl_xor(acc[j], 32, 64);
  }
  if (rl == 0) {
#pragma unroll
    for (int j = 0; j < V; ++j) sacc[wave][cl * V + j] = acc[j];
  }
  __syncthreads();
  if (threadIdx.x < W) {
    const int64_t col = (int64_t)blockIdx.x * W + threadIdx.x;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kColWaves; ++w) s += sacc[w][threadIdx.x];
    if (col < cols) publish(part + (int64_t)blockIdx.y * cols + col, s);
  }
  if (!take_last_ticket(tickets + blockIdx.x, gridDim.y)) return;
  if (threadIdx.x < W) {
    const int64_t col = (int64_t)blockIdx.x * W + threadIdx.x;
    if (col < cols) out[col] = (TO)(fold_chunks(part, (int)gridDim.y, cols, col) * scale);
  }
  if (threadIdx.x == 0) rearm(tickets + blockIdx.x);
}

template <typename T, typename TO>
__global__ __launch_bounds__(256) void rowsum(const T* __restrict__ x, int64_t rows, int64_t cols, int64_t ld,
                                              TO* __restrict__ out, double scale) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const T* p = x + row * ld;
  double acc = 0.0;
  for (int64_t c = lane; c < cols; c += 64) acc += to_f64<T>(p[c]);
  acc = wave_reduce<kRedSum>(acc);
  if (lane == 0) out[row] = (TO)(acc * scale);
}

// 16-B vectors: a wave reads 1 KiB of its row per step (bf16: 512 columns)
template <typename T, typename TO>
__global__ __launch_bounds__(256) void rowsum_v(const T* __restrict__ x, int64_t rows, int64_t cols, int64_t ld,
                                                TO* __restrict__ out, double scale) {
  constexpr int V = 16 / sizeof(T);
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const V16<T>* p = reinterpret_cast<const V16<T>*>(x + row * ld);
  const int64_t nv = cols / V;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int64_t c = lane;
  for (; c + 192 < nv; c += 256) {  // four vectors in flight per lane
    const V16<T> u = p[c], w = p[c + 64], y = p[c + 128], z = p[c + 192];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      a0 += to_f64<T>(u.v[j]);
      a1 += to_f64<T>(w.v[j]);
      a2 += to_f64<T>(y.v[j]);
      a3 += to_f64<T>(z.v[j]);
    }
  }
  for (; c < nv; c += 64) {
    const V16<T> u = p[c];
#pragma unroll
    for (int j = 0; j < V; ++j) a0 += to_f64<T>(u.v[j]);
  }
  const double acc = wave_reduce<kRedSum>((a0 + a1) + (a2 + a3));
  if (lane == 0) out[row] = (TO)(acc * scale);
}

template <typename T, typename TO>
int launch_axis(const T* x, int64_t rows, int64_t cols, int64_t ld, int axis, TO* out, double scale, double* ws,
                hipStream_t s) {
  constexpr int V = 16 / sizeof(T);
  if (axis == 1) {
    if (cols % V == 0 && ld % V == 0 && ((uintptr_t)x & 15) == 0)
      rowsum_v<T, TO><<<(unsigned)((rows + 3) / 4), 256, 0, s>>>(x, rows, cols, ld, out, scale);
    else
      rowsum<T, TO><<<(unsigned)((rows + 3) / 4), 256, 0, s>>>(x, rows, cols, ld, out, scale);
    return launch_status();
  }
  // (strips of 16*V columns while the tickets go round; wider matrices take
  // the scalar kernel's 256-column blocks)
  const bool vec = cols % V == 0 && ld % V == 0 && ((uintptr_t)x & 15) == 0 &&
                   (cols + 16 * V - 1) / (16 * V) <= kAxisTickets;
  const int64_t col_blocks = vec ? (cols + 16 * V - 1) / (16 * V) : (cols + 255) / 256;
  // row chunks: the scalar kernel aims at ~1k blocks of >= 32 rows; the
  // 16-wave vector kernel at ~128 blocks of >= 1024 rows (a block that
  // streams only 2 steps is mostly block start-up, ticket and fold).  4096^2
  // bf16, rocprofv3 min: 1024 blocks x 128 rows 14.2 us, 256 x 512 10.6,
  // 128 x 1024 9.4 (profiles/archive/r3_colsum_chunking_sweep.log,
  // tools/probe/axis_shapes.py).  BK_COLSUM_BLOCKS / BK_COLSUM_MIN_ROWS
  // override the vector targets (lab sweeps).
  static const int64_t vec_blocks = env_int("BK_COLSUM_BLOCKS", 128);
  static const int64_t vec_min_rows = env_int("BK_COLSUM_MIN_ROWS", 1024);
  int64_t chunks = (vec ? vec_blocks : 1024) / col_blocks;
  if (chunks * cols > kAxisWsDoubles) chunks = kAxisWsDoubles / cols;
  const int64_t min_rows = vec ? vec_min_rows : 32;
  if (chunks > (rows + min_rows - 1) / min_rows) chunks = (rows + min_rows - 1) / min_rows;
  if (chunks < 1) chunks = 1;
  const int64_t per = (rows + chunks - 1) / chunks;
  chunks = (rows + per - 1) / per;
  unsigned* tickets = reinterpret_cast<unsigned*>(ws + kAxisWsDoubles);
  if (col_blocks > kAxisTickets) return kBadArgument;
  const dim3 grid((unsigned)col_blocks, (unsigned)chunks);
  if (vec)
    colsum_tile_v<T, TO><<<grid, kColWaves * 64, 0, s>>>(x, rows, cols, ld, per, ws, tickets, out, scale);
  else
    colsum_1pass<T, TO><<<grid, 256, 0, s>>>(x, rows, cols, ld, per, ws, tickets, out, scale);
  return launch_status();
}

}  // namespace bk

using namespace bk;

// sum (op 0) or square-sum (op 1) of the uniform [lo, hi) draw of n values
// at (seed, offset) -- without materialising it.  dtype kF64 or kF32.
BK_API int bk_rand_reduce(int op, int dtype, int64_t n, uint64_t seed, uint64_t offset, double lo, double hi,
                          void* workspace, void* out, hipStream_t stream) {
  if (!workspace || !out || n < 0 || (op != kRedSum && op != kRedSquareSum) || (dtype != kF64 && dtype != kF32))
    return kBadArgument;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const int64_t units = dtype == kF64 ? (n + 1) / 2 : (n + 3) / 4;
  // fixed grid for a given n: results are reproducible run to run
  // (BK_RANDRED_BLOCKS: lab override of the grid cap, <= kRedMaxBlocks)
  static const int64_t max_blocks = env_int("BK_RANDRED_BLOCKS", kRandRedMaxBlocks) <= kRedMaxBlocks
                                        ? env_int("BK_RANDRED_BLOCKS", kRandRedMaxBlocks)
                                        : kRandRedMaxBlocks;
  unsigned g = stream_grid(units > 0 ? (units + 7) / 8 : 1, kRedBlock, (int)(max_blocks / kNumCU));
  if (g > (unsigned)max_blocks) g = (unsigned)max_blocks;
  double* ws = (double*)workspace;
  unsigned* t = reinterpret_cast<unsigned*>(ws + kRedMaxBlocks);
  double* o = (double*)out;
  if (dtype == kF64) {
    if (op == kRedSum) rand_reduce_f64<kRedSum><<<g, kRedBlock, 0, stream>>>(n, k0, k1, offset, lo, hi - lo, ws, t, o);
    else rand_reduce_f64<kRedSquareSum><<<g, kRedBlock, 0, stream>>>(n, k0, k1, offset, lo, hi - lo, ws, t, o);
  } else {
    if (op == kRedSum)
      rand_reduce_f32<kRedSum><<<g, kRedBlock, 0, stream>>>(n, k0, k1, offset, (float)lo, (float)(hi - lo), ws, t, o);
    else
      rand_reduce_f32<kRedSquareSum><<<g, kRedBlock, 0, stream>>>(n, k0, k1, offset, (float)lo, (float)(hi - lo), ws, t,
                                                                  o);
  }
  return launch_status();
}

// partials, then the completion ticket (its own 256 B)
BK_API int bk_reduce_workspace_bytes() { return kRedMaxBlocks * (int)sizeof(double) + 256; }

// A fresh workspace's tickets must read zero (each launch re-arms its own).
BK_API int bk_reduce_workspace_init(void* workspace, hipStream_t stream) {
  if (!workspace) return kBadArgument;
  if (hipMemsetAsync((char*)workspace + kRedMaxBlocks * sizeof(double), 0, 256, stream) != hipSuccess)
    return kLaunchFailed;
  return kOk;
}

// out: ONE double on the device.  workspace: bk_reduce_workspace_bytes() bytes.
// b is only read for kRedDot and kRedMaxAbsDiff (same length and dtype as a).
BK_API int bk_reduce(int op, int dtype, const void* a, const void* b, int64_t n, void* workspace, void* out,
                     hipStream_t stream) {
  if (!a || !out || !workspace || n < 0 || op < 0 || op >= kRedCount || ((op == kRedDot || op == kRedMaxAbsDiff) && !b)) return kBadArgument;
  using Ops = std::make_integer_sequence<int, kRedCount>;
  switch (dtype) {
    case kF64: return dispatch_reduce<double>(op, a, b, n, (double*)workspace, (double*)out, stream, Ops{});
    case kF32: return dispatch_reduce<float>(op, a, b, n, (double*)workspace, (double*)out, stream, Ops{});
    case kBF16: return dispatch_reduce<uint16_t>(op, a, b, n, (double*)workspace, (double*)out, stream, Ops{});
  }
  return kBadArgument;
}

BK_API int64_t bk_reduce_axis_workspace_bytes() {
  return kAxisWsDoubles * (int64_t)sizeof(double) + kAxisTickets * (int64_t)sizeof(unsigned);
}

BK_API int bk_reduce_axis_workspace_init(void* ws, hipStream_t stream) {
  if (!ws) return kBadArgument;
  if (hipMemsetAsync((char*)ws + kAxisWsDoubles * sizeof(double), 0, kAxisTickets * sizeof(unsigned), stream) !=
      hipSuccess)
    return kLaunchFailed;
  return kOk;
}

// out[cols] (axis 0) or out[rows] (axis 1) = sum (op 0) or mean (op 1) of
// x[rows x cols] (row stride ld).  out dtype: f64 for f64 input, f32 for f32
// and bf16 input (f64 accumulation throughout).  ws: the axis workspace.
BK_API int bk_reduce_axis(int op, int dtype, const void* x, int64_t rows, int64_t cols, int64_t ld, int axis, void* out,
                          void* ws, hipStream_t stream) {
  if (!x || !out || !ws || rows <= 0 || cols <= 0 || ld < cols || (axis != 0 && axis != 1) || (op != 0 && op != 1))
    return kBadArgument;
  if (axis == 0 && cols > kAxisWsDoubles) return kBadArgument;  // > 262144 columns: reduce a transposed view instead
  const double scale = op == 1 ? 1.0 / (double)(axis == 0 ? rows : cols) : 1.0;
  double* w = (double*)ws;
  switch (dtype) {
    case kF64: return launch_axis<double, double>((const double*)x, rows, cols, ld, axis, (double*)out, scale, w, stream);
    case kF32: return launch_axis<float, float>((const float*)x, rows, cols, ld, axis, (float*)out, scale, w, stream);
    case kBF16: return launch_axis<uint16_t, float>((const uint16_t*)x, rows, cols, ld, axis, (float*)out, scale, w, stream);
  }
  return kBadArgument;
}
