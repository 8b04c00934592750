// bf16 GEMM, 256x256 block tile, phase-pipelined: C = alpha * A . Bt^T (+ beta C)
//
// Geometry: 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128x64
// output (8x4 fragments of v_mfma_f32_16x16x32_bf16 = 128 accumulator
// registers).  BK = 64.  One block per CU (4096^2 -> 256 blocks = the chip).
//
// LDS (one __shared__ array, 128 KiB): two K-tile buffers, each split into
// four 16 KiB half-tiles of 128 rows x 64 k:
//   A0 = rows {0..63, 128..191} of the A tile   (the "upper" 64 rows of each
//   A1 = rows {64..127, 192..255}                M wave-group)
//   B0 = cols {0..31, 64..95, 128..159, 192..223} of the tile (left 32 of
//   B1 = the other 32 of each wave's 64            every wave's 64 columns)
// so a wave's output quadrant (m-half mh, n-half nh) reads exactly half Amh
// and half Bnh.
//
// Each K-tile runs as 4 phases, one output quadrant (4x2 fragments, K = 64 =
// 16 MFMAs) per phase, in the order (0,0) (0,1) (1,1) (1,0) so consecutive
// phases share an operand held in registers.  Every load is a 16-B
// global_load_lds; the loop never waits for vmcnt(0), and raw s_barrier
// replaces __syncthreads() so prefetches stay in flight across barriers
// (cdna_hip_programming §5 "Pipelining across barriers").  The M wave-group 1
// runs one barrier behind group 0 (an extra s_barrier at entry, matched by
// one at exit), so on every SIMD one wave's MFMAs overlap the other wave's
// fragment reads and prefetch issue.
//
// Two prefetch schedules (template parameter KEEP_B0):
//
// * KEEP_B0 = false (round-1 kernel).  Fragment reads per phase: A0+B0,
//   B1, A1, B0 again.  Last LDS use of a half: A0 @P1, B1 @P2, A1 @P3,
//   B0 @P4; prefetches P1: A1(t+1)  P2: B0(t+1)  P3: A0(t+2)  P4: B1(t+2),
//   one counted `s_waitcnt vmcnt(4)` in P4.  B0(t+1) gets only 2 phases of
//   latency before that wait.
// * KEEP_B0 = true.  The B0 fragments read in P1 stay in 16 extra VGPRs for
//   P4, so B0's slot is free after P1 like A0's.  Prefetches
//   P1: A1(t+1)  P3: A0(t+2) B0(t+2)  P4: B1(t+2): every half-tile is
//   issued >= 5 phases before its first read.  Waits: P2 retires A1(t)
//   (needed in P3), P4 retires A0/B0/B1(t+1) (needed in P1/P2 of t+1); in
//   steady state 8 glds stay in flight per wave through both waits.
//
// Ordering, both schedules (with the stagger):
//   RAW: a half read in phase p+1 was waited for (vmcnt, by every issuing
//        wave) before phase p's first barrier of the issuing group; the
//        reader passes that barrier (group 1's first barrier of p is group
//        0's second) before its phase p+1 reads.
//   WAR: a slot is overwritten >= 2 phases after its last read: reads of
//        phase p retire (compiler lgkmcnt before the MFMAs) before the
//        reading group's second barrier of p.
//
// LDS bank conflicts: rows are 128 B, 16-B chunk c of row r is stored at
// chunk c ^ ((r >> 1) & 7); the swizzle is applied to the per-lane GLOBAL
// source address (global_load_lds writes lane-linear) and undone on the
// ds_read address, which makes each 16-lane ds_read_b128 group (16 rows, one
// logical chunk) hit 16 distinct 16-B bank slots.
//
// Included by gemm_bf16_256.hip (the shipped instantiation) and by
// tools/gemm_lab/gemm_lab.hip (A/B of schedule variants in one binary).
#pragma once
#include "bk_common.hpp"

namespace bk {
namespace g256 {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef const __attribute__((address_space(1))) void* global_void_ptr;

constexpr int TM = 256, TN = 256, TK = 64;
constexpr int kThreads = 512;
constexpr int kHalf = 128 * TK;      // elements per half-tile (16 KiB)
constexpr int kBuf = 4 * kHalf;      // A0 A1 B0 B1
constexpr int kGroupM = 4;           // tiles along M sharing a B panel in L2
// epilogue staging: per wave a 64x64 f32 block, row pitch 68 floats -- the
// 16x16 C/D map writes rows 4q+r (q = lane>>4) at 16 consecutive columns, and
// 4*68*4 B = 16 banks apart makes those four rows hit disjoint banks
constexpr int kEpPitch = 68;
constexpr int kEpWaveFloats = 64 * kEpPitch;
constexpr int kSmemBytes = (2 * kBuf * 2 > 8 * kEpWaveFloats * 4) ? 2 * kBuf * 2 : 8 * kEpWaveFloats * 4;

// Kernel options (compile-time bit set).
enum : int {
  kKeepB0 = 1,    // schedule above
  kStagger = 2,   // run M wave-group 1 one barrier behind group 0
  kSameTile = 4,  // DIAGNOSTIC ONLY: every block reads tile (0,0) -> L2-resident operands, wrong C
};
constexpr int kOptRound1 = kStagger;
constexpr int kOptKeepB0 = kKeepB0 | kStagger;

__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
  const int xcd = b % kNumXCD, q = nblocks / kNumXCD, r = nblocks % kNumXCD;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + b / kNumXCD;
}

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// tile row (A) / tile column (B) held in row r of half h
template <bool IS_A, int H>
__device__ __forceinline__ int half_to_tile(int r) {
  if constexpr (IS_A) return (r >> 6) * 128 + H * 64 + (r & 63);
  else return (r >> 5) * 64 + H * 32 + (r & 31);
}

// One half-tile: 16 wave-instructions of 1 KiB (8 rows) each, 2 per wave.
template <bool IS_A, int H>
__device__ __forceinline__ void stage_half(const uint16_t* __restrict__ g, int ld, int row0, int k0, uint16_t* lds_half,
                                           int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ins = wave * 2 + i;
    const int r = ins * 8 + (lane >> 3);
    const int c = swz(r, lane & 7);
    const uint16_t* src = g + (int64_t)(row0 + half_to_tile<IS_A, H>(r)) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((global_void_ptr)src, (lds_void_ptr)(lds_half + ins * 8 * TK), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag(const uint16_t* lds_half, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds_half + row * TK + swz(row, chunk) * 8);
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct Ctx {
  const uint16_t* A;
  const uint16_t* Bt;
  int lda, ldb, m0, n0, wave, lane, wr, wc;
};

// issue half-tile `which` (0=A0 1=A1 2=B0 3=B1) of K-tile kt into buffer buf
template <int WHICH>
__device__ __forceinline__ void prefetch(const Ctx& c, uint16_t* smem, int buf, int kt) {
  uint16_t* dst = smem + buf * kBuf + WHICH * kHalf;
  if constexpr (WHICH < 2) stage_half<true, WHICH>(c.A, c.lda, c.m0, kt * TK, dst, c.wave, c.lane);
  else stage_half<false, WHICH - 2>(c.Bt, c.ldb, c.n0, kt * TK, dst, c.wave, c.lane);
}

template <int MH>
__device__ __forceinline__ void read_a(const uint16_t* buf, int wr, int lane, bf16x8 (&af)[4][2]) {
  const uint16_t* h = buf + MH * kHalf;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i][s] = frag(h, wr * 64 + i * 16 + (lane & 15), s * 4 + (lane >> 4));
}

template <int NH>
__device__ __forceinline__ void read_b(const uint16_t* buf, int wc, int lane, bf16x8 (&bf)[2][2]) {
  const uint16_t* h = buf + (2 + NH) * kHalf;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) bf[j][s] = frag(h, wc * 32 + j * 16 + (lane & 15), s * 4 + (lane >> 4));
}

template <int MH, int NH>
__device__ __forceinline__ void mfma_quadrant(f32x4 (&acc)[8][4], const bf16x8 (&af)[4][2], const bf16x8 (&bf)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[MH * 4 + i][NH * 2 + j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bf[j][s], acc[MH * 4 + i][NH * 2 + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

template <bool OUT_BF16>
__device__ __forceinline__ void epilogue(const Ctx& c, uint16_t* smem, const f32x4 (&acc)[8][4], void* __restrict__ C,
                                         int ldc, float alpha, float beta) {
  // through LDS (free now: the last barrier retired every read and no
  // prefetch is in flight), so global stores are whole 128-B row segments
  // instead of 2-byte scatters.  Each wave owns its own staging block: no
  // barrier between its LDS writes and reads (same-wave LDS ops are ordered).
  const int lane = c.lane;
  float* ep = reinterpret_cast<float*>(smem) + c.wave * kEpWaveFloats;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ep[(ii * 16 + (lane >> 4) * 4 + r) * kEpPitch + j * 16 + (lane & 15)] = alpha * acc[mh * 4 + ii][j][r];
    const int64_t grow0 = c.m0 + c.wr * 128 + mh * 64;
    const int gcol0 = c.n0 + c.wc * 64;
    if constexpr (OUT_BF16) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = it * 8 + (lane >> 3), col = (lane & 7) * 8;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(ep + row * kEpPitch + col);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(ep + row * kEpPitch + col + 4);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        uint4* dst = reinterpret_cast<uint4*>((uint16_t*)C + (grow0 + row) * ldc + gcol0 + col);
        if (beta != 0.f) {
          const uint4 old = *dst;
          const uint32_t w[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] += beta * bf16_bits_to_float((uint16_t)(w[e] & 0xffff));
            v[2 * e + 1] += beta * bf16_bits_to_float((uint16_t)(w[e] >> 16));
          }
        }
        uint32_t packed[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          packed[e] = (uint32_t)float_to_bf16_bits(v[2 * e]) | ((uint32_t)float_to_bf16_bits(v[2 * e + 1]) << 16);
        *dst = make_uint4(packed[0], packed[1], packed[2], packed[3]);
      }
    } else {
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int row = it * 4 + (lane >> 4), col = (lane & 15) * 4;
        f32x4 v = *reinterpret_cast<const f32x4*>(ep + row * kEpPitch + col);
        f32x4* dst = reinterpret_cast<f32x4*>((float*)C + (grow0 + row) * ldc + gcol0 + col);
        if (beta != 0.f) v += beta * *dst;
        *dst = v;
      }
    }
  }
}

template <bool OUT_BF16, int O>
__global__ __launch_bounds__(kThreads, 1) void gemm_bf16_tn_256(const uint16_t* __restrict__ A,
                                                                const uint16_t* __restrict__ Bt, void* __restrict__ C,
                                                                int M, int N, int K, int lda, int ldb, int ldc,
                                                                float alpha, float beta) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[kSmemBytes / 2];  // 136 KiB, the only LDS object

  const int nbm = M / TM, nbn = N / TN, nblocks = nbm * nbn;
  const int b = xcd_remap(blockIdx.x, nblocks);
  const int group = kGroupM * nbn;
  const int first_m = (b / group) * kGroupM;
  const int gm = min(nbm - first_m, kGroupM);
  const int tm = first_m + (b % group) % gm, tn = (b % group) / gm;

  Ctx c;
  c.A = A;
  c.Bt = Bt;
  c.lda = lda;
  c.ldb = ldb;
  c.m0 = tm * TM;
  c.n0 = tn * TN;
  c.lane = threadIdx.x & 63;
  c.wave = threadIdx.x >> 6;
  c.wr = c.wave >> 2;
  c.wc = c.wave & 3;
  const int lane = c.lane, wr = c.wr, wc = c.wc;
  constexpr bool keep_b0 = (O & kKeepB0) != 0, stagger = (O & kStagger) != 0, same_tile = (O & kSameTile) != 0;
  if constexpr (same_tile) {  // loads of every block hit tile (0,0); stores stay at the block's own tile
    c.A = A - (int64_t)c.m0 * lda;
    c.Bt = Bt - (int64_t)c.n0 * ldb;
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / TK;
  bf16x8 af[4][2], bf[2][2];

  if constexpr (!keep_b0) {
    // prologue: all of tile 0, then the halves of tile 1 that the steady
    // state would have issued in the previous tile's P3/P4
    prefetch<0>(c, smem, 0, 0);
    prefetch<2>(c, smem, 0, 0);
    prefetch<3>(c, smem, 0, 0);
    prefetch<1>(c, smem, 0, 0);
    if (nk > 1) {
      prefetch<0>(c, smem, 1, 1);
      prefetch<3>(c, smem, 1, 1);
      wait_vm<4>();
    } else {
      wait_vm<0>();
    }
    barrier();
    if (stagger && wr == 1) barrier();

    for (int t = 0; t < nk; ++t) {
      const int cur = t & 1, nxt = cur ^ 1;
      const uint16_t* buf = smem + cur * kBuf;
      const bool pf1 = t + 1 < nk, pf2 = t + 2 < nk;

      // P1: quadrant (0,0) -- A0, B0
      read_b<0>(buf, wc, lane, bf);
      read_a<0>(buf, wr, lane, af);
      if (pf1) prefetch<1>(c, smem, nxt, t + 1);
      barrier();
      mfma_quadrant<0, 0>(acc, af, bf);
      barrier();

      // P2: quadrant (0,1) -- B1 (A0 in registers)
      read_b<1>(buf, wc, lane, bf);
      if (pf1) prefetch<2>(c, smem, nxt, t + 1);
      barrier();
      mfma_quadrant<0, 1>(acc, af, bf);
      barrier();

      // P3: quadrant (1,1) -- A1 (B1 in registers)
      read_a<1>(buf, wr, lane, af);
      if (pf2) prefetch<0>(c, smem, cur, t + 2);
      barrier();
      mfma_quadrant<1, 1>(acc, af, bf);
      barrier();

      // P4: quadrant (1,0) -- B0 again (A1 in registers)
      read_b<0>(buf, wc, lane, bf);
      if (pf2) {
        prefetch<3>(c, smem, cur, t + 2);
        wait_vm<4>();  // tile t+1 resident; t+2 in flight
      } else {
        wait_vm<0>();
      }
      barrier();
      mfma_quadrant<1, 0>(acc, af, bf);
      barrier();
    }
  } else {
    bf16x8 b0[2][2];
    // prologue: tile 0 in first-read order, then tile 1's A0/B0 (steady
    // state: previous tile's P3) and B1 (P4); wait as the P4 rule does
    prefetch<0>(c, smem, 0, 0);
    prefetch<2>(c, smem, 0, 0);
    prefetch<3>(c, smem, 0, 0);
    prefetch<1>(c, smem, 0, 0);
    if (nk > 1) {
      prefetch<0>(c, smem, 1, 1);
      prefetch<2>(c, smem, 1, 1);
      prefetch<3>(c, smem, 1, 1);
      wait_vm<8>();  // A0 B0 B1 of tile 0 retired; A1(0) + 3 halves of tile 1 in flight
    } else {
      wait_vm<2>();  // only A1(0) may stay in flight
    }
    barrier();
    if (stagger && wr == 1) barrier();

    for (int t = 0; t < nk; ++t) {
      const int cur = t & 1, nxt = cur ^ 1;
      const uint16_t* buf = smem + cur * kBuf;
      const bool pf1 = t + 1 < nk, pf2 = t + 2 < nk;

      // P1: quadrant (0,0) -- A0, B0 (B0 kept for P4); issue A1(t+1)
      read_b<0>(buf, wc, lane, b0);
      read_a<0>(buf, wr, lane, af);
      if (pf1) prefetch<1>(c, smem, nxt, t + 1);
      barrier();
      mfma_quadrant<0, 0>(acc, af, b0);
      barrier();

      // P2: quadrant (0,1) -- B1; retire A1(t) for P3
      read_b<1>(buf, wc, lane, bf);
      if (pf1) wait_vm<8>();  // younger: A0 B0 B1 A1 of tile t+1
      else wait_vm<0>();
      barrier();
      mfma_quadrant<0, 1>(acc, af, bf);
      barrier();

      // P3: quadrant (1,1) -- A1; slots A0/B0 of this buffer are free
      read_a<1>(buf, wr, lane, af);
      if (pf2) {
        prefetch<0>(c, smem, cur, t + 2);
        prefetch<2>(c, smem, cur, t + 2);
      }
      barrier();
      mfma_quadrant<1, 1>(acc, af, bf);
      barrier();

      // P4: quadrant (1,0) -- B0 from registers; retire A0/B0/B1(t+1)
      if (pf2) {
        prefetch<3>(c, smem, cur, t + 2);
        wait_vm<8>();  // younger: A1(t+1), A0 B0 B1(t+2)
      } else if (pf1) {
        wait_vm<2>();  // younger: A1(t+1)
      } else {
        wait_vm<0>();
      }
      barrier();
      mfma_quadrant<1, 0>(acc, af, b0);
      barrier();
    }
  }
  if (stagger && wr == 0) barrier();  // match group 1's extra barrier
  epilogue<OUT_BF16>(c, smem, acc, C, ldc, alpha, beta);
}

inline bool ok(int M, int N, int K, int lda, int ldb, int ldc, bool out_bf16) {
  // 16-B epilogue stores need 16-B aligned C rows
  return M > 0 && N > 0 && K > 0 && M % TM == 0 && N % TN == 0 && K % TK == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldc % (out_bf16 ? 8 : 4) == 0;
}

template <int O>
inline void launch(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
                   float beta, bool out_bf16, hipStream_t stream) {
  const unsigned grid = (unsigned)((M / TM) * (N / TN));
  if (out_bf16)
    gemm_bf16_tn_256<true, O><<<grid, kThreads, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K, lda,
                                                             ldb, ldc, alpha, beta);
  else
    gemm_bf16_tn_256<false, O><<<grid, kThreads, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K, lda,
                                                              ldb, ldc, alpha, beta);
}

}  // namespace g256
}  // namespace bk
