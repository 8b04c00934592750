// Full-precision GEMM for numpy's own dtypes: C = op(A) . op(B) in f64 on
// v_mfma_f64_16x16x4_f64 and in f32 on v_mfma_f32_16x16x4_f32 (gfx950).
//
// Why this kernel exists: the reference's payloads are plain f64 numpy
// (/root/reference/examples/benchmark-numpy.py:18-22, using_imports.py:20-36);
// the bf16 MFMA GEMM (gemm_bf16.hip) would round them, which numpy never
// does.  Both MFMAs here are exact in their dtype: each is a k-ordered
// chain of fused multiply-adds with one rounding per product (f32: bitwise
// an fmaf chain, cdna_hip_programming.md §3 "FP32-input MFMA"), so the error
// against an fp64 reference is that of a blocked dot product in the dtype.
//
// Hardware budget (MI355X_MICROARCH.md, Matrix cores): the f64 MFMA issues one
// 16x16x4 product (2048 flop) per 64 cycles per SIMD and the f32 one per 32
// cycles -- 78.6 / 157.3 TFLOP/s dense over 256 CUs.  Both are slow next to
// the LDS and L2, so the design goal is simply to keep every SIMD issuing
// MFMAs back to back:
//
//  * workgroup tile 64 x 64 (64 x 32 for mid-size products), 4 waves of
//    32 x 32 (2 x 2 accumulators of 16x16) per K group; a k-step of 4 is 2 A
//    + 2 B one-element fragment reads for 4 MFMAs, and the next k-step's
//    reads are issued before this one's MFMAs (fragment lookahead);
//  * K tile 16 deep (128 B per f64 row, 64 B per f32 row), two LDS stages,
//    one barrier per K tile; global -> registers -> LDS through two register
//    stages, so three K tiles of 16-B loads are in flight;
//  * the loads go through one buffer descriptor per operand panel: rows and
//    K columns past the matrix read as zero in hardware, so edge tiles, the
//    partial K tile and the loop's tail run the same branch-free code as the
//    interior (the f64 kernel needs 106 VGPRs, four workgroups per CU);
//  * LDS holds each operand tile in its global orientation (rows copied as
//    16-B chunks), padded so the fragment reads are bank-conflict free in
//    either orientation -- so A^T / B^T views (numpy's a.T, e.g. np.dot(a.T,
//    a)) are read in place, no transpose pass;
//  * XCD-aware tile order: blocks land on XCD b % 8, so each XCD gets a
//    contiguous run of tiles, walked in groups of 4 tile rows (the A row
//    panels and B column panels a group shares stay in that XCD's L2).
//
// Small products (at most ~1.5 64 x 64 tiles per CU) run two K groups per
// workgroup whose halves meet in LDS (deterministic, no C memset).  128-row
// tiles remain for A/B runs only (profiles/r6_gemm_fp_pmc.md).
//
// Any M, N, K and leading dimensions: 16-B buffer loads when the pointers,
// leading dimensions and K allow them; otherwise guarded 16-B / element loads
// (out-of-range elements zero).  Stores are masked.
#include "bk_common.hpp"

namespace bk {
namespace fp {

// The MFMA steps of a K tile (0-3) before which the next tile is staged:
// its LDS stores before step 1, the global loads that refill its registers
// before step 2 -- mid-tile, between MFMAs, not in one burst with the tile's
// first fragment reads.  Both at step 2 was 1.6% faster (geometric mean over
// f64 / f32 1536-4096^3) than both at the top (session r6_s29); splitting
// them 1 / 2 another 0.8% (2 / 3 0.5%, 1 / 3 level: session r6_s39;
// profiles/r6_gemm_fp_sweep.jsonl).  -D for A/B builds.
#ifndef BK_FP_STORE_AT
#define BK_FP_STORE_AT 1
#endif
#ifndef BK_FP_LOAD_AT  // (the refill loads' step, >= BK_FP_STORE_AT)
#define BK_FP_LOAD_AT 2
#endif
// The tile order walks groups of this many tile rows (their A panels, and
// the B panels the group shares, stay in the XCD's L2): 4 -- 0.8% faster than
// 8 over f64 / f32 2048-8192^3 (f64 8192^3 15730 vs 16262 us), 16 2% slower,
// 2 1.75% slower, 1 4.5% (sessions r6_s45, r6_s47).  -D for A/B builds.
#ifndef BK_FP_GROUP
#define BK_FP_GROUP 4
#endif
constexpr int kBM = 128, kThreads = 256;  // (kBM: the A/B runs' 128-row tiles)

// An [m|n][k] LDS row is padded by 2 elements: 16 B for f64, 8 B for f32
// (with 16 B the f32 fragment reads' ds_read2_b32 pairs put rows r and r + 8
// on one bank; 8 B: bank conflicts / LDS-active 0.33 -> 0.14 at 2048^3 and
// 0.5-1.5% faster at every size, profiles/r6_gemm_fp_sweep.jsonl "pad8").
// (Splitting the pairs into single ds_read_b32 / _b64 reads measured slower
// everywhere: 2048^3 f32 164 vs 143 us, f64 303 vs 277; the pairs halve the
// LDS instructions and their address arithmetic.)
template <typename T>
struct Cfg {
  static constexpr int pitch_k(int bk) { return bk + 2; }
};

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <typename T>
using acc_t = typename std::conditional<std::is_same<T, double>::value, f64x4, f32x4>::type;

__device__ __forceinline__ f64x4 mfma(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Accumulator element r of lane l -> (row, col) in the 16x16 tile.  The f64
// MFMA has its own C/D map (cdna_hip_programming.md §3, Fragment layout):
// the f32 row formula on it puts 3 of every 4 results in the wrong row.
template <typename T>
__device__ __forceinline__ int acc_row(int lane, int r) {
  if constexpr (std::is_same<T, double>::value)
    return (lane >> 4) + 4 * r;
  else
    return (lane >> 4) * 4 + r;
}

// One operand tile: `ROWS` x `COLS` elements of a row-major buffer starting
// at (r0, c0), copied to LDS in the same orientation as 16-B chunks (LDS row
// pitch PITCH elements).  An A tile is BM x BK ([m][k]) or BK x BM ([k][m]);
// a B tile BK x BN or BN x BK.  Chunks are spread evenly over the 256 threads
// of one K group (`tid`; consecutive threads take consecutive chunks of a row:
// every 16-B load of a wave lands in whole 64-B segments); a tile of fewer
// chunks than threads (16 x 32 f32) leaves the last threads idle.
template <typename T, bool VEC, int ROWS, int COLS, int PITCH>
struct Tile {
  static constexpr int E = 16 / sizeof(T);  // elements per 16-B chunk
  static constexpr int CPR = COLS / E;      // chunks per tile row
  static constexpr int kTotal = ROWS * CPR;
  static constexpr int kChunks = (kTotal + kThreads - 1) / kThreads;
  static constexpr bool kPartial = kTotal % kThreads != 0;
  static_assert(!kPartial || kTotal < kThreads, "whole chunks per thread, or one chunk for some threads");
  static constexpr int kLdsElems = ROWS * PITCH;
  static_assert(kLdsElems * sizeof(T) % 16 == 0, "16-B aligned LDS stages");
  T v[kChunks][E];

  __device__ __forceinline__ static bool owns(int q) { return !kPartial || q < kTotal; }

  // every element in range (an interior tile): 16-B loads, no guards
  __device__ __forceinline__ void load_fast(const T* __restrict__ g, int64_t ld, int r0, int c0, int tid) {
    const T* base = g + (int64_t)r0 * ld + c0;
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
      const int q = c * kThreads + tid;
      if (!owns(q)) continue;
      const u32x4_t w = *reinterpret_cast<const u32x4_t*>(base + (int64_t)(q / CPR) * ld + (q % CPR) * E);
      __builtin_memcpy(v[c], &w, 16);
    }
  }

  // Through a buffer descriptor whose range (num_records) ends the panel:
  // rows past it read as zero, and so do chunks at or past column `col_lim`
  // (their offset is moved out of range: the caller passes the K extent
  // when the tile's columns run along K, so a partial K tile and the
  // K tiles past the end are zeros).  No branches: every tile, edges
  // included, loads the same way (BUF).  (r0, c0) are panel-relative.
  __device__ __forceinline__ void load_buf(__amdgpu_buffer_rsrc_t rsrc, int64_t ld, int r0, int c0, int col_lim,
                                           int tid) {
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
      const int q = c * kThreads + tid;
      if (!owns(q)) continue;
      const int row = r0 + q / CPR, col = c0 + (q % CPR) * E;
      const int off = col < col_lim ? (int)(((int64_t)row * ld + col) * (int64_t)sizeof(T)) : (int)0x80000000;
      const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
      __builtin_memcpy(v[c], &x, 16);
    }
  }

  // edge tiles: out-of-range elements are zero
  __device__ __forceinline__ void load_guarded(const T* __restrict__ g, int64_t ld, int row_end, int col_end, int r0,
                                               int c0, int tid) {
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
      const int q = c * kThreads + tid;
      if (!owns(q)) continue;
      const int row = r0 + q / CPR, col = c0 + (q % CPR) * E;
      const T* p = g + (int64_t)row * ld + col;
      if (VEC && row < row_end && col + E <= col_end) {
        const u32x4_t w = *reinterpret_cast<const u32x4_t*>(p);
        __builtin_memcpy(v[c], &w, 16);
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) v[c][e] = (row < row_end && col + e < col_end) ? p[e] : T(0);
      }
    }
  }

  __device__ __forceinline__ void store(T* lds, int tid) const {
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
      const int q = c * kThreads + tid;
      if (!owns(q)) continue;
      T* dst = lds + (q / CPR) * PITCH + (q % CPR) * E;
      if constexpr (PITCH * sizeof(T) % 16 == 0) {
        u32x4_t w;
        __builtin_memcpy(&w, v[c], 16);
        *reinterpret_cast<u32x4_t*>(dst) = w;
      } else {  // (8-B aligned rows)
        uint64_t w[2];
        __builtin_memcpy(w, v[c], 16);
        reinterpret_cast<uint64_t*>(dst)[0] = w[0];
        reinterpret_cast<uint64_t*>(dst)[1] = w[1];
      }
    }
  }
};

// C[M][N] = A . B, A[m][k] at a[TA ? k*lda + m : m*lda + k], B[k][n] at
// b[TB ? n*ldb + k : k*ldb + n].  Workgroup tile BM x BN (64 x 64 / 64 x 32;
// 128 x 64 / 128 x 128 for A/B runs); 4 waves of BM/2 x BN/2 per K group.
//
// KS = 2 (small products): two K groups of 4 waves each take one half of the
// K tiles with their own LDS stages, and at the end group 1 hands its
// accumulators to group 0 through LDS: C = fl(p0 + p1) in one fixed order, so
// the product is deterministic with no C memset, no atomics and no
// workspace.  (It replaces a two-way split over separate workgroups that
// added both halves into a zeroed C with float atomics; that memset alone was
// 5 us of a 36 us 1024^3 f32 product, profiles/r6_gemm_fp_pmc.md.)
//
// RS register stages of global loads (RS = 2: three K tiles of loads in
// flight), PIPE fragment lookahead (below).  su > 0 staggers the K loop:
// workgroup b starts at K tile ((b % su) * ss) of its range and wraps (L2 /
// HBM channel spread, rocBLAS's "StaggerU"; measured level here, so off by
// default).  A group whose range ends in a partial K tile takes that tile
// first instead, in the prologue, so every later load is a whole tile.  The
// K order is fixed per output tile: the result is deterministic.
template <typename T, bool TA, bool TB, bool VEC, int BM, int BN, int BK, int OCC, int KS, int RS, bool PIPE,
          bool BUF = false>
__global__ __launch_bounds__(kThreads * KS, OCC) void gemm_fp_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                                    T* __restrict__ c, int M, int N, int K,
                                                                    int64_t lda, int64_t ldb, int64_t ldc,
                                                                    const unsigned* __restrict__ gate, int su, int ss) {
  // gated launch (the split-bf16 f32 product's fallback, bk_gemm_f32x6):
  // runs only when the split found operands it cannot represent
  if (gate && *gate == 0) return;
  constexpr int PK = Cfg<T>::pitch_k(BK);
  constexpr int MI = BM / 32, kPitchM = BM + 16;  // MI 16-row blocks per wave
  constexpr int kPitchN = BN + 16;  // a [k][n] row: f64 = 32, f32 = 16 dwords mod 64 banks
  constexpr int WN = BN / 2, NT = WN / 16;  // wave columns, 16-wide MFMA tiles per wave row
  static_assert(NT >= 1 && MI >= 1 && BK % 4 == 0, "tile");
  // A tile: [m][k] (row-major A) or [k][m] (A^T view); B tile: [k][n] or [n][k]
  using TileA = typename std::conditional<TA, Tile<T, VEC, BK, BM, kPitchM>, Tile<T, VEC, BM, BK, PK>>::type;
  using TileB = typename std::conditional<TB, Tile<T, VEC, BN, BK, PK>, Tile<T, VEC, BK, BN, kPitchN>>::type;
  // LDS: per K group two stages of (A tile, B tile); KS = 2 reuses it for the
  // hand-over of group 1's accumulators (4 waves x MI x NT x 4 x 64 values)
  constexpr int kStage = TileA::kLdsElems + TileB::kLdsElems;
  constexpr int kXchg = KS > 1 ? 4 * MI * NT * 4 * 64 : 0;
  constexpr int kSmem = KS * 2 * kStage > kXchg ? KS * 2 * kStage : kXchg;
  __shared__ __attribute__((aligned(16))) T smem[kSmem];

  // ---- tile of this block (XCD-aware, grouped) ----
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int total = tiles_m * tiles_n;
  const int raw = (int)blockIdx.x;
  // XCD-aware order: blocks are dealt round-robin over the 8 XCDs, so XCD x
  // runs blocks x, x+8, ...; they get a contiguous range of tiles (the first
  // total % 8 XCDs one more), whose A / B panels then share that XCD's L2
  const int per_xcd = total / kNumXCD, extra = total % kNumXCD, xcd = raw % kNumXCD;
  const int bid = xcd * per_xcd + min(xcd, extra) + raw / kNumXCD;
  constexpr int kGroup = BK_FP_GROUP;  // tile rows walked together (their A panels shared in L2)
  const int per_group = kGroup * tiles_n;
  const int first_m = (bid / per_group) * kGroup;
  const int gsz = min(tiles_m - first_m, kGroup);
  const int tm = first_m + (bid % per_group) % gsz, tn = (bid % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const bool interior = VEC && m0 + BM <= M && n0 + BN <= N;  // (uniform)

  const int grp = KS > 1 ? (int)threadIdx.x / kThreads : 0;  // K group (wave-uniform)
  const int tid = (int)threadIdx.x % kThreads;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * WN;
  const int fr = lane & 15, fk = lane >> 4;  // fragment: row/col within 16, k within 4

  acc_t<T> acc[MI][NT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = acc_t<T>{0, 0, 0, 0};

  TileA ta[RS];
  TileB tb[RS];
  auto load_fast = [&](auto slot, int k0) {
    constexpr int q = decltype(slot)::value;
    if constexpr (TA)
      ta[q].load_fast(a, lda, k0, m0, tid);
    else
      ta[q].load_fast(a, lda, m0, k0, tid);
    if constexpr (TB)
      tb[q].load_fast(b, ldb, n0, k0, tid);
    else
      tb[q].load_fast(b, ldb, k0, n0, tid);
  };
  // BUF: one buffer descriptor per operand panel -- A's rows m0.. ([m][k])
  // or its columns m0.. over all K rows ([k][m]), B's columns n0.. over all K
  // rows ([k][n]) or its rows n0.. ([n][k]) -- whose range ends at the
  // matrix's last element, so rows past M / N / K read as zero
  // (launch() checks every panel offset fits 31 bits)
  // (num_records is 32 bits: a panel of 2 GiB or more -- the rest of a big
  // matrix from this tile's first row -- is capped at 2^31 - 1, which every
  // in-range offset stays below (launch()'s fits()); cast unclamped, 4 GiB
  // and up would wrap to a short range and read real rows as zero)
  auto panel = [](const T* base, int64_t elems) {
    const int64_t bytes = elems * (int64_t)sizeof(T);
    const int64_t cap = 0x7fffffffll;
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(bytes < 0 ? 0 : bytes > cap ? cap : bytes),
                                             0x00020000);
  };
  const __amdgpu_buffer_rsrc_t ra =
      TA ? panel(a + m0, (int64_t)(K - 1) * lda + M - m0) : panel(a + (int64_t)m0 * lda, (int64_t)(M - m0 - 1) * lda + K);
  const __amdgpu_buffer_rsrc_t rb =
      TB ? panel(b + (int64_t)n0 * ldb, (int64_t)(N - n0 - 1) * ldb + K) : panel(b + n0, (int64_t)(K - 1) * ldb + N - n0);
  constexpr int kNoLim = 0x7fffffff;
  auto load = [&](auto slot, int k0) {
    constexpr int q = decltype(slot)::value;
    if constexpr (BUF) {
      // (columns past M / N of the [k][m] / [k][n] views read neighbours'
      // values: they only feed C's rows / columns past the edge, never stored)
      if constexpr (TA)
        ta[q].load_buf(ra, lda, k0, 0, kNoLim, tid);
      else
        ta[q].load_buf(ra, lda, 0, k0, K, tid);
      if constexpr (TB)
        tb[q].load_buf(rb, ldb, 0, k0, K, tid);
      else
        tb[q].load_buf(rb, ldb, k0, 0, kNoLim, tid);
    } else if (interior && k0 + BK <= K) {
      load_fast(slot, k0);
    } else {
      if constexpr (TA)
        ta[q].load_guarded(a, lda, K, M, k0, m0, tid);
      else
        ta[q].load_guarded(a, lda, M, K, m0, k0, tid);
      if constexpr (TB)
        tb[q].load_guarded(b, ldb, N, K, n0, k0, tid);
      else
        tb[q].load_guarded(b, ldb, K, N, k0, n0, tid);
    }
  };
  T* const stage0 = smem + grp * 2 * kStage;
  auto lds_a = [&](int st) { return stage0 + st * kStage; };
  auto lds_b = [&](int st) { return stage0 + st * kStage + TileA::kLdsElems; };

  // Pipeline (two LDS stages, RS register stages, loads 1 + RS K tiles
  // ahead): iteration kt stores tile kt+1 -- in registers since iteration
  // kt-RS -- into the other LDS stage (last read in iteration kt-1, before
  // the barrier that ended it), then issues tile kt+1+RS's global loads into
  // the freed registers, while it runs tile kt's MFMAs (before steps
  // BK_FP_STORE_AT / BK_FP_LOAD_AT; the edge-tile variant at the top of the
  // iteration).
  const int nk_all = (K + BK - 1) / BK, nk_per = (nk_all + KS - 1) / KS;
  const int kt0 = grp * nk_per;                      // this group's K tiles: [kt0, kt0 + nk)
  const int nk = max(0, min(nk_per, nk_all - kt0));  // (group 1 may have one fewer, or none)
  const bool partial = K % BK != 0 && kt0 + nk == nk_all;
  const int rot = nk <= 0 ? 0 : partial ? nk - 1 : su > 0 ? (int)(((int64_t)(raw % su) * ss) % nk) : 0;
  auto kpos = [&](int t) {  // K offset of this group's t-th tile
    if (BUF && t >= nk) return nk_all * BK;  // (BUF: past the group's range, a tile of zeros)
    int r = t + rot;
    if (r >= nk) r -= nk;
    return (kt0 + r) * BK;
  };
  using S0 = std::integral_constant<int, 0>;
  if (BUF || nk > 0) {
    load(S0{}, kpos(0));
    ta[0].store(lds_a(0), tid);
    tb[0].store(lds_b(0), tid);
    // tiles 1 .. RS into register slots t % RS
    if (BUF || nk > 1) load(std::integral_constant<int, 1 % RS>{}, kpos(1));
    if constexpr (RS > 1)
      if (BUF || nk > 2) load(S0{}, kpos(2));
  }
  __syncthreads();

  // Fragment lookahead (PIPE): the fragments of MFMA step s+1 are read from
  // LDS while step s's MFMAs run, and the next K tile's step 0 right after
  // the iteration's one barrier, which sits before the last step's MFMAs.
  // Without it every step read its fragments and waited for them
  // (lgkmcnt(0)) before its MFMAs: f64 2048^3 waves spent 120K cycles in
  // s_waitcnt against the Tensile kernel's 22K of the same 64 x 64 x 16 tile
  // (profiles/r6_gemm_fp_pmc.md).
  constexpr int kSteps = BK / 4;
  T pa[MI], pb[NT];
  auto read_frag = [&](const T* As, const T* Bs, int kk, T(&fa)[MI], T(&fb)[NT]) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = wm + i * 16 + fr, k = kk + fk;
      fa[i] = TA ? As[k * kPitchM + m] : As[m * PK + k];
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = wn + j * 16 + fr, k = kk + fk;
      fb[j] = TB ? Bs[n * PK + k] : Bs[k * kPitchN + n];
    }
  };
  if constexpr (PIPE)
    if (nk > 0) read_frag(lds_a(0), lds_b(0), 0, pa, pb);

  // An interior tile (`fast`) takes a branch-free variant: every iteration
  // stores and loads (past the last tile it re-loads tile nk-1, a whole one,
  // into a stage nobody reads), so the loads of the register slots stay in
  // flight together -- with the guarded, branchy loads the compiler's wait
  // before each LDS store drains every slot (vmcnt(0)).
  const bool fast = BUF || ((PIPE || RS > 1) && interior && nk == nk_per && (!partial || nk >= 2));
  auto step = [&](int kt, auto slot, auto fast_tag) __attribute__((always_inline)) {  // slot = (kt + 1) % RS
    constexpr int q = decltype(slot)::value;
    constexpr bool kFast = decltype(fast_tag)::value;
    const int cur = kt & 1;
    auto store_next = [&]() {
      ta[q].store(lds_a(cur ^ 1), tid);
      tb[q].store(lds_b(cur ^ 1), tid);
    };
    auto load_next = [&]() {
      if constexpr (BUF)
        load(slot, kpos(kt + 1 + RS));  // (past the end: zero tiles)
      else
        load_fast(slot, kpos(min(kt + 1 + RS, nk - 1)));
    };
    constexpr int kStoreAt = PIPE ? BK_FP_STORE_AT : 0;
    constexpr int kLoadAt = PIPE ? BK_FP_LOAD_AT : 0;
    static_assert(kLoadAt >= kStoreAt, "a slot's loads follow its LDS stores");
    if constexpr (kFast) {
      if constexpr (kStoreAt == 0) store_next();
      if constexpr (kLoadAt == 0) load_next();
    } else {
      if (kt >= nk) {  // (group 1's surplus iteration: only the barrier)
        __syncthreads();
        return;
      }
      if (kt + 1 < nk) {
        ta[q].store(lds_a(cur ^ 1), tid);
        tb[q].store(lds_b(cur ^ 1), tid);
        if (kt + 1 + RS < nk) load(slot, kpos(kt + 1 + RS));
      }
    }
    const T* As = lds_a(cur);
    const T* Bs = lds_b(cur);
    if constexpr (PIPE) {
#pragma unroll
      for (int s4 = 0; s4 < kSteps; ++s4) {
        if constexpr (kFast && kStoreAt > 0)
          if (s4 == kStoreAt) store_next();
        if constexpr (kFast && kLoadAt > 0)
          if (s4 == kLoadAt) load_next();
        T ca[MI], cb[NT];
#pragma unroll
        for (int i = 0; i < MI; ++i) ca[i] = pa[i];
#pragma unroll
        for (int j = 0; j < NT; ++j) cb[j] = pb[j];
        if (s4 + 1 < kSteps) {
          read_frag(As, Bs, 4 * (s4 + 1), pa, pb);
        } else {
          // every wave stored tile kt+1 at the top of this iteration and
          // issued its last reads of stage cur: the stages swap here
          __syncthreads();
          if (kFast || kt + 1 < nk) read_frag(lds_a(cur ^ 1), lds_b(cur ^ 1), 0, pa, pb);
        }
        // (keeps the reads ahead of this step's MFMAs: the scheduler would
        // sink them below, and the wait for them would then follow at once)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma(ca[i], cb[j], acc[i][j]);
      }
    } else {
      // (the 128 x 128 tile: no registers for a lookahead set)
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        T fa[MI], fb[NT];
        read_frag(As, Bs, kk, fa, fb);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
      }
      __syncthreads();
    }
  };
  // (both variants run nk_per iterations: the K groups meet at every barrier)
  auto run = [&](auto fast_tag) {
    // (the loop body runs both register slots' steps unconditionally and an
    // odd last step follows it: with the second step conditional inside the
    // loop, the path that skipped it reached the first step's LDS stores with
    // one slot of loads in flight, and the compiler's wait there drained both
    // slots on every path -- vmcnt(0) every other K tile.  1024^3 / 1536^3
    // 1-2.5% faster, larger sizes level: profiles/r6_gemm_fp_sweep.jsonl,
    // session r6_s30)
    int kt = 0;
    for (; kt + RS <= nk_per; kt += RS) {
      step(kt, std::integral_constant<int, 1 % RS>{}, fast_tag);
      if constexpr (RS > 1) step(kt + 1, S0{}, fast_tag);
    }
    if constexpr (RS > 1)
      if (kt < nk_per) step(kt, std::integral_constant<int, 1 % RS>{}, fast_tag);
  };
  // (BUF: one branch-free loop for every tile; the guarded variant and its
  // registers are not in the kernel at all -- f64 64 x 64: 112 VGPRs
  // against 152, a fourth workgroup per CU)
  if constexpr (BUF) {
    run(std::true_type{});
  } else {
    if (fast)
      run(std::true_type{});
    else
      run(std::false_type{});
  }

  if constexpr (KS > 1) {
    // group 1 -> LDS -> group 0 (the loop's last barrier ended every LDS read
    // that counts; lookahead reads after it are discarded);
    // value (i, j, r) of lane l of wave w at ((((w * MI + i) * NT + j) * 4 + r) * 64 + l):
    // each store / load instruction covers 64 consecutive values
    __syncthreads();
    T* x = smem + (int64_t)wave * (MI * NT * 4 * 64) + lane;
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) x[((i * NT + j) * 4 + r) * 64] = acc[i][j][r];
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += x[((i * NT + j) * 4 + r) * 64];
  }

  // ---- epilogue: lanes 0..15 of a row are 16 consecutive columns ----
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm + i * 16 + acc_row<T>(lane, r);
      if (m >= M) continue;
      T* crow = c + (int64_t)m * ldc;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n0 + wn + j * 16 + fr;
        if (n < N) crow[n] = acc[i][j][r];
      }
    }
  }
}

struct LaunchArgs {
  const void *A, *B;
  void* C;
  int M, N, K;
  int64_t lda, ldb, ldc;
  hipStream_t stream;
  const unsigned* gate;
  int su, ss;
  unsigned grid;
  bool buf;  // the branch-free buffer-load kernels (BUF) take this product
};

template <typename T, bool TA, bool TB, bool V, int BM, int BN, int BK, int OCC, int KS, int RS, bool PIPE>
void go(const LaunchArgs& g) {
  if constexpr (V) {
    if (g.buf) {
      gemm_fp_kernel<T, TA, TB, true, BM, BN, BK, OCC, KS, RS, PIPE, true><<<g.grid, kThreads * KS, 0, g.stream>>>(
          (const T*)g.A, (const T*)g.B, (T*)g.C, g.M, g.N, g.K, g.lda, g.ldb, g.ldc, g.gate, g.su, g.ss);
      return;
    }
  }
  gemm_fp_kernel<T, TA, TB, V, BM, BN, BK, OCC, KS, RS, PIPE><<<g.grid, kThreads * KS, 0, g.stream>>>(
      (const T*)g.A, (const T*)g.B, (T*)g.C, g.M, g.N, g.K, g.lda, g.ldb, g.ldc, g.gate, g.su, g.ss);
}

struct Shape {
  int bm, bn, ks, rs;
};

// 64-row tiles (64 or 32 wide, one or two K groups) or 128-row ones (64 or
// 128 wide); two register stages and the fragment lookahead everywhere but
// the 128 x 128 tile, whose registers have no room for either (f64: 241
// VGPRs of 256; f32 at three per CU: spills past 168)
template <typename T, bool TA, bool TB, bool V, int BK, int OCC>
void by_shape(const LaunchArgs& g, const Shape& s) {
  constexpr bool kF64 = std::is_same<T, double>::value;
  if (s.bm == 64) {
    if (s.bn == 32 && s.ks == 2)
      go<T, TA, TB, V, 64, 32, BK, OCC, 2, 2, true>(g);
    else if (s.bn == 32)
      s.rs == 2 ? go<T, TA, TB, V, 64, 32, BK, OCC, 1, 2, true>(g) : go<T, TA, TB, V, 64, 32, BK, OCC, 1, 1, true>(g);
    else if (s.ks == 2)
      s.rs == 2 ? go<T, TA, TB, V, 64, 64, BK, OCC, 2, 2, true>(g) : go<T, TA, TB, V, 64, 64, BK, OCC, 2, 1, true>(g);
    else
      s.rs == 2 ? go<T, TA, TB, V, 64, 64, BK, OCC, 1, 2, true>(g) : go<T, TA, TB, V, 64, 64, BK, OCC, 1, 1, true>(g);
  } else if constexpr (!(kF64 && BK == 32)) {  // (f64 32-deep: 64-row tiles only)
    if (s.bn == 64)
      s.rs == 2 ? go<T, TA, TB, V, 128, 64, BK, OCC, 1, 2, true>(g) : go<T, TA, TB, V, 128, 64, BK, OCC, 1, 1, true>(g);
    else
      go<T, TA, TB, V, 128, 128, BK, OCC, 1, 1, false>(g);
  }
}

// Tile shape and depth (profiles/r6_gemm_fp_sweep.jsonl).  For A/B runs
// (tools/gemm_fp_bench.py, tools/gemm_fp_sweep.sh) the choice can be
// overridden: BK_GEMM_FP_BN (32 | 64 | 128 columns), BK_GEMM_FP_BM (64 | 128
// rows), BK_GEMM_FP_KS (1 | 2 K groups), BK_GEMM_FP_RS (1 | 2 register
// stages), BK_GEMM_FP_BK (f32: 16 | 32 deep), BK_GEMM_FP_SU / _SS (stagger),
// BK_GEMM_FP_TINY=0 (no 64 x 32 split for the smallest grids),
// BK_GEMM_FP_BUF=0 (guarded loads only).
template <typename T, bool TA, bool TB>
void launch(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, bool vec,
            hipStream_t stream, const unsigned* gate = nullptr) {
  constexpr bool kF64 = std::is_same<T, double>::value;
  auto env = [](const char* name, int dflt) {
    const char* v = getenv(name);
    return v ? atoi(v) : dflt;
  };
  const int64_t t64 = (int64_t)((M + 63) / 64) * ((N + 63) / 64);
  // 64-row tiles (profiles/r6_gemm_fp_pmc.md, "Tile shapes with the buffer
  // loads": the 128-row tiles lost at every size once the buffer-load kernels
  // let a CU hold four 64 x 64 f64 workgroups, eight f32 ones -- f32 3072^3
  // 423 vs 578 us with 128 x 128):
  //  * at most half a 64 x 64 tile per CU: 64 x 32 tiles with two K groups,
  //    twice the workgroups of the 64 x 64 split (f64 512^3 13.5 vs 21.2 us,
  //    640^3 16.4 vs 25.2; f32 512^3 9.3 vs 13.3 -- session r6_s38; from
  //    768^3 it lost, r6_s34);
  //  * at most one 64 x 64 tile per CU: two K groups per workgroup (1024^3:
  //    256 tiles; f64 47 vs 51 us with one group; past one per CU a second
  //    round of these 8-wave workgroups lost to 64 x 32 tiles, 1152^3 79.3
  //    vs 65.2 us -- session r6_s41);
  //  * 64 x 32 tiles where they share the work out over the CUs clearly more
  //    evenly: `fill` is the busy share of the CUs when every CU takes
  //    ceil(tiles / CUs) tiles, and a 64 x 32 tile does less work per loaded
  //    byte, so it must gain > 0.1 of it (1536^3 0.90 vs 0.75: f64 143 vs
  //    166 us; 1792^3 0.875 vs 0.77: 211 vs 223; 1280^3 0.78 both: 64 x 64,
  //    92 vs 99; 2560^3 0.96 vs 0.89: 64 x 64, 530 vs 548 --
  //    profiles/r6_gemm_fp_sweep.jsonl, sessions r6_s24, r6_s35);
  //  * 64 x 64 everywhere else.
  auto fill = [](int64_t n) {
    const int64_t per = (n + kNumCU - 1) / kNumCU;
    return per > 0 ? (double)n / (double)(per * kNumCU) : 1.0;
  };
  // (f32: two K groups come with the 32-deep K tile below, so they need K >= 512)
  const int nk_split = kF64 ? (K + 15) / 16 : (K + 31) / 32;
  Shape s{64, 64, 1, 2};
  if (2 * t64 <= kNumCU && nk_split >= 16 && env("BK_GEMM_FP_TINY", 1) != 0)
    s = {64, 32, 2, 2};
  else if (t64 <= kNumCU && nk_split >= 16)
    s = {64, 64, 2, 2};
  else if (fill(2 * t64) > fill(t64) + 0.1)
    s = {64, 32, 1, 2};
  s.bm = env("BK_GEMM_FP_BM", s.bm) == 64 ? 64 : kBM;
  s.bn = env("BK_GEMM_FP_BN", s.bn);
  if (s.bn != 32 && s.bn != 64) s.bn = 128;
  if (s.bm == 64 && s.bn == 128) s.bn = 64;  // (64-row tiles come 64 or 32 wide)
  if (s.bm == kBM && s.bn == 32) s.bn = 64;  // (and 128-row ones 64 or 128)
  s.ks = s.bm == 64 && s.bn <= 64 && env("BK_GEMM_FP_KS", s.ks) == 2 ? 2 : 1;
  s.rs = env("BK_GEMM_FP_RS", s.rs) == 1 ? 1 : 2;
  // K tile 16 deep; f32 32 deep on the small products' shapes -- two K
  // groups or 64 x 32 tiles -- where it halves the barriers (1024^3 25.2 vs
  // 26.0 us, 1536^3 75.3 vs 76.4), 16 on 64 x 64 tiles, whose halved LDS
  // lets a CU hold more workgroups (1280^3 51.3 vs 52.5; sessions r6_s32,
  // r6_s35)
  const int bk = env("BK_GEMM_FP_BK", !kF64 && (s.ks == 2 || s.bn == 32) ? 32 : 16) == 32 ? 32 : 16;
  const int64_t tiles = (int64_t)((M + s.bm - 1) / s.bm) * ((N + s.bn - 1) / s.bn);
  // BUF (branch-free buffer loads, the guarded path compiled out) when the
  // 16-B chunks along K are all in or all out (K a multiple of the chunk)
  // and every panel offset -- rows up to a tile past the edge -- fits 31 bits
  // (two K groups too since the register-slot loop keeps a slot in flight:
  // f32 1024^3 23.6 vs 24.2 us, 768^3 18.2 vs 18.8, f64 level; before it
  // they were slower, 50.3 vs 48.1 -- sessions r6_s23, r6_s37)
  constexpr int kE = 16 / (int)sizeof(T);
  auto fits = [](int64_t rows, int64_t ld) { return (rows + 256) * ld * (int64_t)sizeof(T) < 0x7fffffffll; };
  const bool buf = vec && K % kE == 0 && env("BK_GEMM_FP_BUF", 1) != 0 &&
                   fits(TA ? K : s.bm, lda) && fits(TB ? s.bn : K, ldb);
  LaunchArgs g{A, B, C, M, N, K, lda, ldb, ldc, stream, gate, env("BK_GEMM_FP_SU", 0), env("BK_GEMM_FP_SS", 1),
               (unsigned)tiles, buf};
  auto depth = [&](auto v) {
    constexpr bool V = decltype(v)::value;
    if constexpr (kF64) {
      if (bk == 32 && s.bm == 64)  // (A/B runs; 128-row f64 tiles have no registers for it)
        by_shape<T, TA, TB, V, 32, 2>(g, s);
      else
        by_shape<T, TA, TB, V, 16, 2>(g, s);
    } else if (bk == 16)
      by_shape<T, TA, TB, V, 16, 3>(g, s);
    else
      by_shape<T, TA, TB, V, 32, 2>(g, s);
  };
  if (vec)
    depth(std::true_type{});
  else
    depth(std::false_type{});
}

template <typename T>
void dispatch(bool ta, bool tb, const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
              int64_t ldc, bool vec, hipStream_t s, const unsigned* gate = nullptr) {
  if (ta && tb)
    launch<T, true, true>(A, B, C, M, N, K, lda, ldb, ldc, vec, s, gate);
  else if (ta)
    launch<T, true, false>(A, B, C, M, N, K, lda, ldb, ldc, vec, s, gate);
  else if (tb)
    launch<T, false, true>(A, B, C, M, N, K, lda, ldb, ldc, vec, s, gate);
  else
    launch<T, false, false>(A, B, C, M, N, K, lda, ldb, ldc, vec, s, gate);
}


// ---- f32 product on the bf16 MFMA: the six-piece split (bk_gemm_f32x6) ----
//
// An f32 value a (24-bit significand) is the exact sum of three bf16 pieces
// (8 bits each): a0 = bf16(a), a1 = bf16(a - a0), a2 = bf16(a - a0 - a1); each
// difference is exact (Sterbenz), so |a - (a0 + a1 + a2)| <= 2^-25 |a|.  A
// product of two pieces has at most 16 significant bits, exact in the bf16
// MFMA's f32 accumulator, and
//   a . b = a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0 + (a1 b2 + a2 b1 + a2 b2)
// where the bracket is below 2^-24 |a b| -- f32's own rounding unit -- and is
// dropped.  So one bf16 GEMM over K' = 6 Kp with
//   A' row = [a0 | a0 | a1 | a0 | a1 | a2],  B' row = [b0 | b1 | b0 | b2 | b1 | b0]
// (each block Kp = K rounded up to 64, zero-padded) gives the f32 product with
// f32-level error (6x the additions of a plain f32 dot product), at the bf16
// MFMA's rate: 6 x 2 x 2.5 PFLOP/s-class passes against f32's 157 TFLOP/s.
//
// The split needs |a| in [2^-100, 2^127) or a == 0: infinities and NaNs
// (inf * a zero piece is NaN), values whose bf16 head overflows, and values
// whose pieces fall below the normal range.  A piece kernel that meets one
// sets the workspace's flag word (cleared first, on the stream); the plain f32
// kernel is then launched gated on that flag and recomputes C only if set.
constexpr uint32_t kSplitPatA = 0 | 0 << 2 | 1 << 4 | 0 << 6 | 1 << 8 | 2 << 10;
constexpr uint32_t kSplitPatB = 0 | 1 << 2 | 0 << 4 | 2 << 6 | 1 << 8 | 0 << 10;
constexpr int kSplitTile = 64;

__device__ __forceinline__ uint32_t bf16_rn_bits(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// three pieces of 8 values, packed 8 bf16 per u32x4; true if any value is
// outside the split's range
__device__ __forceinline__ bool split8(const float (&x)[8], u32x4_t (&p)[3]) {
  bool bad = false;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    uint32_t w[3] = {0, 0, 0};
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float a = x[2 * h + e];
      const float m = fabsf(a);
      bad |= !(m < 0x1p127f) || (m != 0.f && m < 0x1p-100f);
      const uint32_t h0 = bf16_rn_bits(a);
      const float r1 = a - __uint_as_float(h0 << 16);
      const uint32_t h1 = bf16_rn_bits(r1);
      const uint32_t h2 = bf16_rn_bits(r1 - __uint_as_float(h1 << 16));
      w[0] |= h0 << (16 * e);
      w[1] |= h1 << (16 * e);
      w[2] |= h2 << (16 * e);
    }
    p[0][h] = w[0];
    p[1][h] = w[1];
    p[2][h] = w[2];
  }
  return bad;
}

// dst[r][j * Kp + k] = piece pat_j of src(r, k) for r < rows, k < Kp (zero past
// K).  COLS: src(r, k) = src[k * ld + r] (an [K][rows] buffer, staged through
// LDS to transpose), else src[r * ld + k].  One 64 x 64 tile per workgroup;
// thread t handles rows t / 8 + 32 q (q = 0, 1) and the 8 k of chunk t % 8,
// so each group of 8 lanes writes 128 contiguous bytes of each block.
template <bool COLS, bool VEC>
__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ src, int rows, int K, int64_t ld, int Kp,
                                                     uint16_t* __restrict__ dst, uint32_t pat,
                                                     unsigned* __restrict__ flag) {
  constexpr int T = kSplitTile, kPitch = T + 1;  // +1: the column reads below hit 64 banks
  __shared__ float tile[COLS ? T * kPitch : 1];
  const int tiles_k = Kp / T;
  const int r0 = (int)(blockIdx.x / tiles_k) * T, k0 = (int)(blockIdx.x % tiles_k) * T;
  const int tid = (int)threadIdx.x, kc = tid & 7;
  const int64_t ldd = 6 * (int64_t)Kp;
  if constexpr (COLS) {
    // 64 k-lines of 64 rows: lane runs of 16 x 4 consecutive rows per line
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kl = (tid >> 4) + 16 * i, rr = (tid & 15) * 4;
      const int k = k0 + kl, r = r0 + rr;
      float v[4];
      if (VEC && k < K && r + 4 <= rows) {
        const f32x4 w = *reinterpret_cast<const f32x4*>(src + (int64_t)k * ld + r);
        v[0] = w[0], v[1] = w[1], v[2] = w[2], v[3] = w[3];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (k < K && r + e < rows) ? src[(int64_t)k * ld + r + e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) tile[kl * kPitch + rr + e] = v[e];
    }
    __syncthreads();
  }
  bool bad = false;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int rl = (tid >> 3) + 32 * q, r = r0 + rl, k = k0 + kc * 8;
    if (r >= rows) continue;
    float x[8];
    if constexpr (COLS) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = tile[(kc * 8 + e) * kPitch + rl];
    } else {
      const float* p = src + (int64_t)r * ld + k;
      if (VEC && k + 8 <= K) {
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(p), w1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = w0[e], x[4 + e] = w1[e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = k + e < K ? p[e] : 0.f;
      }
    }
    u32x4_t pc[3];
    bad |= split8(x, pc);
    uint16_t* o = dst + (int64_t)r * ldd + k;
#pragma unroll
    for (int j = 0; j < 6; ++j) *reinterpret_cast<u32x4_t*>(o + (int64_t)j * Kp) = pc[(pat >> (2 * j)) & 3];
  }
  // (rare: a vector atomic from the lanes that found one)
  if (bad) atomicOr(flag, 1u);
}

}  // namespace fp
}  // namespace bk

using namespace bk;

// C[M][N] = op(A) . op(B) in f64 (dtype kF64) or f32 (kF32), row-major C with
// leading dimension ldc.  trans_a: A is given as its transpose, a [K][M]
// buffer (lda >= M); else [M][K] (lda >= K).  trans_b: B given as a [N][K]
// buffer (ldb >= K); else [K][N] (ldb >= N).  Never reads C.
BK_API int bk_gemm_fp(int dtype, int trans_a, int trans_b, const void* A, const void* B, void* C, int M, int N, int K,
                      int64_t lda, int64_t ldb, int64_t ldc, hipStream_t stream) {
  if (dtype != kF64 && dtype != kF32) return kBadArgument;
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0) return kBadArgument;
  if (lda < (trans_a ? M : K) || ldb < (trans_b ? K : N) || ldc < N) return kBadArgument;
  const int64_t tiles = (int64_t)((M + 63) / 64) * ((N + 31) / 32);  // (the smallest tiles: 64 x 32)
  if (tiles > 0x7fffffffll) return kBadArgument;
  const int es = dtype_size(dtype);
  const int e = 16 / es;
  const bool vec = ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % e == 0 && ldb % e == 0;
  if (dtype == kF64)
    fp::dispatch<double>(trans_a != 0, trans_b != 0, A, B, C, M, N, K, lda, ldb, ldc, vec, stream);
  else
    fp::dispatch<float>(trans_a != 0, trans_b != 0, A, B, C, M, N, K, lda, ldb, ldc, vec, stream);
  return launch_status();
}


// ---- C = op(A) . op(B) for f32 operands on the bf16 MFMA GEMM, f32-level
// error (the six-piece split above).  Same operand conventions as
// bk_gemm_fp.  `ws` (16-B aligned, bk_gemm_f32x6_workspace_bytes) holds a
// flag word and the split operands A' [M][6 Kp], B' [N][6 Kp].  Operands the
// split cannot represent (inf / NaN, |x| >= 2^127, 0 < |x| < 2^-100) make the
// plain f32 kernel recompute C, gated on the flag (no host sync).
BK_API int bk_gemm_bf16_tn(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                           float alpha, float beta, int out_dtype, hipStream_t stream);

static int64_t f32x6_kp(int K) { return ((int64_t)K + fp::kSplitTile - 1) / fp::kSplitTile * fp::kSplitTile; }

BK_API int64_t bk_gemm_f32x6_workspace_bytes(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  return 256 + 12 * f32x6_kp(K) * ((int64_t)M + N);
}

BK_API int bk_gemm_f32x6(int trans_a, int trans_b, const void* A, const void* B, void* C, int M, int N, int K,
                         int64_t lda, int64_t ldb, int64_t ldc, void* ws, int64_t ws_bytes, hipStream_t stream) {
  if (!A || !B || !C || !ws || M <= 0 || N <= 0 || K <= 0) return kBadArgument;
  if (lda < (trans_a ? M : K) || ldb < (trans_b ? K : N) || ldc < N || ldc > 0x7fffffffll) return kBadArgument;
  const int64_t kp = f32x6_kp(K);
  // the bf16 kernels' int K / leading dimensions and 31-bit tile extents
  if (6 * kp > (1 << 22) || ws_bytes < bk_gemm_f32x6_workspace_bytes(M, N, K) || (uintptr_t)ws % 16) return kBadArgument;
  unsigned* flag = (unsigned*)ws;
  // the header (flag word + padding) is written, so every workspace byte is
  // (the broker's lazy scrub counts on that for an exactly-sized workspace)
  if (hipMemsetAsync(ws, 0, 256, stream) != hipSuccess) return kLaunchFailed;
  uint16_t* a6 = (uint16_t*)((char*)ws + 256);
  uint16_t* b6 = a6 + 6 * kp * (int64_t)M;
  auto split = [&](bool cols, const void* src, int rows, int64_t ld, uint16_t* dst, uint32_t pat) {
    const bool vec = (uintptr_t)src % 16 == 0 && ld % 4 == 0;
    const unsigned grid = (unsigned)(((rows + fp::kSplitTile - 1) / fp::kSplitTile) * (kp / fp::kSplitTile));
    const float* s = (const float*)src;
    if (cols && vec)
      fp::split3_kernel<true, true><<<grid, 256, 0, stream>>>(s, rows, K, ld, (int)kp, dst, pat, flag);
    else if (cols)
      fp::split3_kernel<true, false><<<grid, 256, 0, stream>>>(s, rows, K, ld, (int)kp, dst, pat, flag);
    else if (vec)
      fp::split3_kernel<false, true><<<grid, 256, 0, stream>>>(s, rows, K, ld, (int)kp, dst, pat, flag);
    else
      fp::split3_kernel<false, false><<<grid, 256, 0, stream>>>(s, rows, K, ld, (int)kp, dst, pat, flag);
  };
  // A(m, k): [M][K] rows, or the [K][M] buffer of an A^T view (columns);
  // B(n, k): the [N][K] buffer of a B^T view (rows), or [K][N] (columns)
  split(trans_a != 0, A, M, lda, a6, fp::kSplitPatA);
  split(trans_b == 0, B, N, ldb, b6, fp::kSplitPatB);
  int rc = launch_status();
  if (rc != kOk) return rc;
  rc = bk_gemm_bf16_tn(a6, b6, C, M, N, (int)(6 * kp), (int)(6 * kp), (int)(6 * kp), (int)ldc, 1.f, 0.f, kF32, stream);
  if (rc != kOk) return rc;
  const bool vec = ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % 4 == 0 && ldb % 4 == 0;
  fp::dispatch<float>(trans_a != 0, trans_b != 0, A, B, C, M, N, K, lda, ldb, ldc, vec, stream, flag);
  return launch_status();
}
