// bf16 GEMM, 256x256 block tile, FOUR waves of 128x128: C = alpha * A . Bt^T (+ beta C)
//
// Why four waves (measured, profiles/archive/r1_gemm_lab.log + PMC): the 8-wave
// 128x64-per-wave kernel (gemm256_impl.hpp) issues 238 ds_read_b128 per CU
// per K-tile and runs 8 barriers per K-tile; its MFMA pipes were busy 58% of
// the cycles, and moving its operands into L2 (diagnostic variant) bought only
// 2%, so the limiter is inside the CU, not HBM.  A 128x128 wave tile reads
// each A row and B column once per 128 outputs instead of per 64: 128
// ds_read_b128 per CU per K-tile (32 per wave), and the whole K-tile needs ONE
// barrier.
//
// Geometry: 256 threads = 4 waves as 2 (M) x 2 (N), one wave per SIMD; each
// wave owns 8x8 fragments of v_mfma_f32_16x16x32_bf16 = 256 accumulator
// registers (the unified VGPR/AGPR file gives one wave 512).  BK = 64.
//
// LDS (one __shared__ array, 128 KiB): two K-tile buffers of [A 256x64 | B
// 256x64] bf16, rows of 128 B with the 16-B chunk XOR swizzle of
// gemm256_impl.hpp (chunk c of row r at c ^ ((r >> 1) & 7): conflict-free
// ds_read_b128), staged by buffer_load ... lds (16 per wave per K-tile)
// through one buffer descriptor per operand panel.
//
// Loop (K-tile t in buffer cur = t & 1, fragments double-buffered in
// registers by k-half s):
//     ds_read  frags(t, s=1)                      [cur]
//     64 MFMA  frags(t, s=0)
//     s_waitcnt lgkmcnt(0) vmcnt(0)               own reads of cur done; own
//     s_barrier                                   glds of t+1 landed
//     glds     tile t+2 -> cur                    WAR-safe: every wave passed
//     ds_read  frags(t+1, s=0)        [nxt]       RAW-safe: every wave's t+1
//     64 MFMA  frags(t, s=1)                      loads retired pre-barrier
// so the MFMA stream only stops at the barrier, every LDS read has 64 MFMAs
// (>= 1024 cycles) to land, and every K-tile load has one whole iteration.
// The only vmcnt(0) in the loop waits for loads issued an iteration earlier.
//
// Shipped options (gemm_bf16_256.hip): kAsmMfma | kInterleave with the
// two-barrier K-loop (kTwoBar | kTwoBarG10, ktile_asm2 below: the wait for
// the next K-tile sits in the second k-half, not at the k-half boundary
// sketched above) and non-temporal C stores (kNtStore).  Inline-asm MFMAs:
// with builtin MFMAs the allocator moved accumulators through
// v_accvgpr_mov in the loop and the kernel lost to the 8-wave one.
#pragma once
#include "bk_common.hpp"

namespace bk {
namespace g4 {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef const __attribute__((address_space(1))) void* global_void_ptr;

constexpr int TM = 256, TN = 256, TK = 64;
constexpr int kThreads = 256;
constexpr int kOperand = 256 * TK;   // elements of one operand's K-tile (32 KiB)
constexpr int kBuf = 2 * kOperand;   // A | B
constexpr int kGroupM = 4;           // tiles along M sharing a B panel in L2
constexpr int kGlds = kOperand / (kThreads * 8);  // glds per wave per operand per K-tile (8)
// epilogue staging: per wave 32 rows x 128 f32, pitch 132 (4 rows of the
// 16x16 C map land 16 banks apart: conflict-free ds_write_b32)
constexpr int kEpPitch = 132;
constexpr int kEpRows = 32;
constexpr int kEpWaveFloats = kEpRows * kEpPitch;
constexpr int kSmemBytes = 2 * kBuf * 2;  // 128 KiB (epilogue needs 66 KiB)
static_assert(4 * kEpWaveFloats * 4 <= kSmemBytes, "epilogue staging fits");

// options
enum : long long {
  kPinOrder = 1,    // sched_barrier fences around each MFMA block
  kInterleave = 2,  // sched_group_barrier: spread ds_read / glds among the MFMAs
  kNoCarry = 4,     // no fragment prefetch across the barrier: both k-halves read at the top of the iteration
  kDirectStore = 8, // epilogue: each lane stores its accumulators straight to C (no LDS staging)
  // MFMAs as inline asm with AGPR-constrained accumulators ("+a"): the 256
  // accumulator registers are pinned in the AGPR file, so the allocator has
  // nothing to shuffle (the builtin form got v_accvgpr_read/write copies in
  // the loop, tools/gemm_lab/isa_check.sh).  The hazard recognizer does not
  // see through inline asm, so accumulator reads after the loop are fenced by
  // explicit wait states (mfma_drain).
  kAsmMfma = 16,
  kEarlyGlds = 32,   // kAsmMfma|kInterleave: all K-tile loads in the first 8 of the second k-half's 16 groups
  kReadsEarly = 64,  // kAsmMfma|kInterleave: k-half-1 fragment reads done by group 11 of 16
  // tile order (lab): M-group size other than kGroupM
  kGroup2 = 128,
  kGroup8 = 256,
  kGroup16 = 512,
  // any M, N, and K % 8 == 0: ceil-div grid, each operand panel's descriptor
  // bounded by the rows that exist (the rest read as zero), chunks past K in
  // the last K-tile read as zero, and blocks on the ragged border -- or any
  // block when ldc breaks the vector stores' alignment -- store element by
  // element under a mask
  kEdge = 1024,
  // B given as [K][N] (C = A . B): transposed LDS reads, see make_panel_nn
  // (tile-multiple shapes, K % 64 == 0)
  kNN = 2048,
  // kAsmMfma|kInterleave with three barriers per K-tile (ktile_asm3): each
  // operand's LDS region is refilled as soon as every wave has its k-half-1
  // fragments of it, and the wait for the next K-tile moves to MFMA 92 of 128
  kThreeBar = 4096,
  // kThreeBar with the 16 K-tile loads spread one per 8 MFMAs (MFMA 24-108)
  // instead of packed into MFMA 24-80: an LDS-DMA issue costs the wave
  // ~60-185 cycles (MI355X_MICROARCH.md), more than one 4-MFMA group
  kSpread = 8192,
  // DIAGNOSTIC (lab only, wrong C): every block but block 0 skips the
  // epilogue, so a timing difference against the same option set without it
  // is the epilogue's cost
  kDiagNoEpilogue = 16384,
  // TN only: MFMAs take the B fragment as srcA (C^T = Bt . A^T per 16x16
  // block) and B's fragment rows are read in a permuted column order, so a
  // lane ends up holding 8 consecutive columns of one C row across the pair of
  // fragments (2p, 2p+1) -- the epilogue stores straight from the
  // accumulators, 16 B per lane, with no LDS staging (epilogue_rows)
  kSwapAB = 32768,
  // the waves on odd SIMDs (HW_ID) run the ktile_asm schedule with each
  // group's LDS/VMEM ops ahead of its 4 MFMAs instead of behind them, so the
  // 4 waves of a CU do not issue their reads and loads in lockstep
  // (hipBLASLt's MT256x256x64 loop has two such orderings, picked the same way)
  kAltSimd = 65536,
  // DIAGNOSTIC (lab only, C overwritten): s_memtime stamps around each
  // K-tile's wait + barrier; every wave writes (loop cycles, cycles in the
  // wait + barrier, K-tiles) as 3 u32 at C + 16 * (block * 4 + wave) bytes
  kDiagStamps = 131072,
  // DIAGNOSTIC (lab only, wrong C): the K-loop issues no glds (the LDS keeps
  // the prologue's two tiles): what the loads cost the MFMA stream
  kDiagNoGlds = 262144,
  // ktile_asm's second k-half: the 16 glds in groups 0-7 (2 each) and the
  // 16 next-tile fragment reads in groups 8-15 (2 each), never in one group
  kSplitGlds = 524288,
  // every group's memory ops pinned between its MFMAs, apart from each
  // other: first k-half M M r M M, second k-half M G M M r M (hipBLASLt's
  // spacing of LDS-DMA loads and LDS reads)
  kSpacedMem = 1048576,
  // DIAGNOSTIC (lab only, wrong C; with kDiagStamps): no LDS reads and no
  // loads in the K-loop -- the MFMA stream alone
  kDiagMfmaOnly = 2097152,
  // kSpacedMem, TN tile multiples: the K-tile's offset moves into each
  // panel's buffer descriptor once per K-tile, every load's SGPR offset is
  // loop-invariant (one SALU fewer per load; hipBLASLt's form)
  kConstSoff = 4194304,
  // kAsmMfma|kInterleave, two barriers per K-tile (ktile_asm2): the wait for
  // the next K-tile's loads in the middle of the second k-half
  kTwoBar = 8388608,
  // kTwoBar: the K-tile wait at group 10 / 12 of the second k-half (default 8)
  kTwoBarG10 = 16777216,
  kTwoBarG12 = 33554432,
  // the LDS-staged epilogue's 16-B stores non-temporal (hipBLASLt's "NTD")
  kNtStore = 67108864,
  // DIAGNOSTICS of kTwoBar (lab only, racy C): drop the K-tile vmcnt wait,
  // the second barrier, or the first lgkmcnt(0) + barrier -- what each costs
  kDiagNoVmWait = 134217728,
  kDiagNoBar2 = 268435456,
  kDiagNoBar1 = 536870912,
  // DIAGNOSTIC of kTwoBar (wrong C): skip the next K-tile's fragment reads
  // (the k-half-0 MFMAs reuse stale fragments); with kDiagNoGlds: no K-loop loads
  kDiagNoReads0 = 1073741824,
  // kTwoBar: the 16 k-half-1 fragment reads over groups 0-11 of the first
  // k-half (2, 2, 2, 2, then 1 per group) instead of 0-7 (2 per group): a
  // lighter LDS read burst next to the landing K-tile loads
  kReads12 = 1LL << 31,
};
// (the stamps' running total while a kDiagStamps kernel runs: one per wave)
struct StampAcc {
  uint64_t wait = 0, h0 = 0, h1 = 0, t_end = 0;  // wait + barrier, k-half 0, k-half 1 (to the next K-tile's start)
};

__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
  const int xcd = b % kNumXCD, q = nblocks / kNumXCD, r = nblocks % kNumXCD;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + b / kNumXCD;
}

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// One operand's 256-row panel as a buffer resource (SRD in SGPRs): loads
// address it with a 2-VGPR per-lane offset + an SGPR offset instead of 16
// 64-bit per-lane pointers, and rows past the panel read as zero.
struct Panel {
  __amdgpu_buffer_rsrc_t rsrc;
  int lane_off[4];  // bytes: (lane/8) rows + this lane's swizzled 16-B chunk, for even / odd i
                    // (kNN B panels: 4 variants, see make_panel_nn)
  int row_bytes;    // ld * 2
  int k_lim[2];     // kEdge: this lane's chunk holds K columns while k0 < k_lim (K - 8 * chunk)
  __attribute__((ext_vector_type(4))) unsigned w;  // kNN: the same descriptor as 4 SGPR words (glds_raw)
};

typedef __attribute__((ext_vector_type(4))) unsigned srd4;

// a raw buffer descriptor's words (what __builtin_amdgcn_make_buffer_rsrc
// builds with stride 0 and these flags), wave-uniform
__device__ __forceinline__ srd4 srd_words(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  srd4 w;
  w.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
  w.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  w.z = __builtin_amdgcn_readfirstlane(bytes);
  w.w = 0x00020000u;
  return w;
}

// buffer_load_dwordx4 ... lds written as inline asm.  The kNN kernel issues
// its direct-to-LDS loads this way because the compiler, seeing an LDS DMA in
// flight, puts an s_waitcnt vmcnt(0) before every ds_read_b64_tr_b16 (whose
// memory operand it cannot disambiguate) -- 14x the wait cycles
// (profiles/archive/r2_gemm_pmc_4096.jsonl).  Hidden from the compiler, the loads are
// ordered by the schedule's own s_waitcnt vmcnt + s_barrier, as before.
__device__ __forceinline__ void glds_raw(const srd4& w, const uint16_t* lds, int voff, int soff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(lds_void_ptr)(lds));
  const int so = __builtin_amdgcn_readfirstlane(soff);
  // s_nop 0: an M0 write followed by an LDS-DMA load needs one wait state
  // (cdna_asm_programming.md §4.1 row 16), which the compiler cannot insert
  // inside the string.  The SGPR operands come from SALU code (no
  // v_readfirstlane in the K-loop: checked in the -save-temps .s), so no
  // VALU-write -> VMEM-read pad is needed ahead of the load.
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(m0), "v"(voff), "s"(w),
               "s"(so)
               : "memory", "m0");
}

__device__ __forceinline__ Panel make_panel(const uint16_t* base, int ld, int lane, int rows = 256, int K = 0) {
  Panel p;
  // descriptor inputs readfirstlane'd so the compiler can PROVE the SRD
  // uniform (else it wraps every load in a waterfall loop: guide T20)
  const uint64_t addr = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)addr);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32));
  // `rows` (< 256 on the ragged border) bounds the panel: the last real row
  // ends at (rows-1)*ld*2 + K*2 <= rows*ld*2, every row past it is out of
  // range and loads zeros
  const int64_t span = (int64_t)rows * ld * 2;  // integer clamp (HIP's min() has no int64 overload: it went through f64)
  const uint32_t bytes = __builtin_amdgcn_readfirstlane(span > 0xffffffffll ? 0xffffffffu : (uint32_t)span);
  p.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
  p.w = srd_words(base, bytes);
  p.row_bytes = ld * 2;
  // row r = wave*64 + i*8 + lane/8 -> swizzle key (r>>1)&7 = (i*4 + lane/16)&7
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int c = (lane & 7) ^ ((par * 4 + (lane >> 4)) & 7);
    p.lane_off[par] = (lane >> 3) * ld * 2 + c * 16;
    p.k_lim[par] = K - c * 8;
  }
  return p;
}

// ---- kNN: B stored [K][N] (row-major, ldb >= N) ------------------------------
// The B K-tile is staged as its own 64 rows (k) x 256 columns (n) of 512 B,
// 32-B units XOR-swizzled by f(row) = (row & 3) | ((row >> 3) & 1) << 2, and
// each MFMA B fragment (8 consecutive k of one n per lane) is read with two
// ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group, delivered
// column-major: cdna_hip_programming.md T10).  Within a 32-lane half the two
// groups read rows 8 apart; f maps the 8 rows to 8 distinct 32-B bank
// windows, so the transposed reads are conflict-free.  glds writes LDS
// lane-linearly, so each lane fetches the global chunk that belongs at its
// LDS slot (the inverse swizzle in its offset).
__device__ __forceinline__ int nn_f(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }

__device__ __forceinline__ Panel make_panel_nn(const uint16_t* base, int ld, int lane, int K) {
  Panel p;
  const uint64_t addr = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)addr);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32));
  const int64_t span = (int64_t)K * ld * 2;
  const uint32_t bytes = __builtin_amdgcn_readfirstlane(span > 0xffffffffll ? 0xffffffffu : (uint32_t)span);
  p.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
  p.w = srd_words(base, bytes);
  p.row_bytes = ld * 2;
  const int b = lane >> 5, pos16 = lane & 31;
  // glds instruction i of a wave fills LDS rows 2*(8*wave + i) + b; f of
  // that row depends on i only through (i & 1) and (i >> 2)
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int i = (v & 1) | ((v >> 1) << 2);
    const int f = ((2 * i + b) & 3) | ((i >> 2) << 2);
    const int u = (pos16 >> 1) ^ f;
    p.lane_off[v] = b * ld * 2 + (u * 2 + (pos16 & 1)) * 16;
  }
  p.k_lim[0] = p.k_lim[1] = 0;
  return p;
}

__device__ __forceinline__ void glds_nn(const Panel& p, int k0, uint16_t* lds_operand, int wave, int i) {
  const int soff = (k0 + (wave * 8 + i) * 2) * p.row_bytes;
  glds_raw(p.w, lds_operand + (wave * kGlds + i) * 8 * TK, p.lane_off[(i & 1) | ((i >> 2) << 1)], soff);
}

// the A operand's glds of a kNN kernel (same addressing as glds_one), raw
__device__ __forceinline__ void glds_a_raw(const Panel& p, int k0, uint16_t* lds_operand, int wave, int i) {
  const int soff = (wave * 64 + i * 8) * p.row_bytes + k0 * 2;
  glds_raw(p.w, lds_operand + (wave * kGlds + i) * 8 * TK, p.lane_off[i & 1], soff);
}

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// B fragment of n-block u (16 columns: u in 0..15 of the 256) for k-half s
__device__ __forceinline__ bf16x8 frag_nn(const uint16_t* lds_b, int u, int s, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  s16x4 v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = s * 32 + 8 * g + 4 * h + q;
    const uint16_t* a = lds_b + row * 256 + ((u ^ nn_f(row)) * 16) + p * 4;
    v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<uint16_t*>(a)));
  }
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const s16x8 w = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
  return __builtin_bit_cast(bf16x8, w);
}

// a lane's 16-B chunk at column k0 + 8 * chunk: past K (the ragged last
// K-tile of kEdge) its offset becomes 2^31, beyond every panel's extent, and
// the load returns zeros.  (K % 8 == 0: chunks are all in or all out.)
// (kt is a compile-time constant at every call: the select folds away
// when false)
__device__ __forceinline__ int chunk_off(const Panel& p, int k0, int par, bool kt) {
  return (kt && k0 >= p.k_lim[par]) ? (int)0x80000000 : p.lane_off[par];
}

// stage one operand's K-tile: 8 wave-instructions of 1 KiB (8 rows) each;
// `wave` must be wave-uniform (readfirstlane'd) so the LDS base goes to M0
__device__ __forceinline__ void stage(const Panel& p, int k0, uint16_t* lds_operand, int wave, bool kt = false,
                                      bool nn = false, bool raw_a = false) {
  if (nn) {
#pragma unroll
    for (int i = 0; i < kGlds; ++i) glds_nn(p, k0, lds_operand, wave, i);
    return;
  }
  if (raw_a) {
#pragma unroll
    for (int i = 0; i < kGlds; ++i) glds_a_raw(p, k0, lds_operand, wave, i);
    return;
  }
#pragma unroll
  for (int i = 0; i < kGlds; ++i) {
    const int soff = (wave * 64 + i * 8) * p.row_bytes + k0 * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(p.rsrc, (lds_void_ptr)(lds_operand + (wave * kGlds + i) * 8 * TK), 16,
                                             chunk_off(p, k0, i & 1, kt), soff, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag(const uint16_t* lds_operand, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds_operand + row * TK + swz(row, chunk) * 8);
}

// B fragment j (columns wc*128 + j*16 ...) of k-half s, either layout
// kSwapAB: fragment j = 2p + h, row rho = lane & 15 holds column
// 32p + 8(rho >> 2) + 4h + (rho & 3), so the MFMA output lane with row group g
// holds columns 32p + 8g + 4h + 0..3
__device__ __forceinline__ int swap_col(int j, int rho) {
  return 32 * (j >> 1) + 8 * (rho >> 2) + 4 * (j & 1) + (rho & 3);
}

__device__ __forceinline__ bf16x8 fragB(const uint16_t* lds_b, int wc, int j, int s, int lane, bool nn,
                                        bool swap = false) {
  if (nn) return frag_nn(lds_b, wc * 8 + j, s, lane);
  if (swap) return frag(lds_b, wc * 128 + swap_col(j, lane & 15), s * 4 + (lane >> 4));
  return frag(lds_b, wc * 128 + j * 16 + (lane & 15), s * 4 + (lane >> 4));
}

// the 8 A (rows wr*128 + i*16 + lane&15) and 8 B fragments of k-half s
__device__ __forceinline__ void read_frags(const uint16_t* buf, int wr, int wc, int lane, int s, bf16x8 (&fa)[8],
                                           bf16x8 (&fb)[8], bool nn = false, bool swap = false) {
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[i] = frag(buf, wr * 128 + i * 16 + (lane & 15), s * 4 + (lane >> 4));
#pragma unroll
  for (int j = 0; j < 8; ++j) fb[j] = fragB(buf + kOperand, wc, j, s, lane, nn, swap);
}

template <bool ASM = false>
__device__ __forceinline__ void mfma_block(f32x4 (&acc)[8][8], const bf16x8 (&fa)[8], const bf16x8 (&fb)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (ASM)
        asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fa[i]), "v"(fb[j]));
      else
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
}

// wait states between the last inline-asm MFMA and any read of its result
// (16x16x32 bf16: 8 passes; 3 x s_nop 7 = 24 wait states covers it)
__device__ __forceinline__ void mfma_drain() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// 64 MFMAs with `ds` ds_reads and `vm` VMEM ops spread evenly among them
template <int DS, int VM>
__device__ __forceinline__ void interleave_hint() {
  constexpr int slots = 16;
#pragma unroll
  for (int q = 0; q < slots; ++q) {
    if constexpr (VM > 0) __builtin_amdgcn_sched_group_barrier(0x020, VM / slots, 0);
    if constexpr (DS > 0) __builtin_amdgcn_sched_group_barrier(0x100, DS / slots, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
  }
}

// one MFMA as inline asm; INIT: C starts from the constant 0
template <bool INIT>
__device__ __forceinline__ void mfma_asm(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (INIT)
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
  else
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// acc (block i, j) += A-fragment i . B-fragment j, in either operand order
template <bool INIT, bool SWAP>
__device__ __forceinline__ void mfma_ab(f32x4& acc, const bf16x8& fa, const bf16x8& fb) {
  if constexpr (SWAP) mfma_asm<INIT>(acc, fb, fa);
  else mfma_asm<INIT>(acc, fa, fb);
}

// the i-th of one operand's 8 K-tile glds (stage() split up)
__device__ __forceinline__ void glds_one(const Panel& p, int k0, uint16_t* lds_operand, int wave, int i,
                                         bool kt = false) {
  const int soff = (wave * 64 + i * 8) * p.row_bytes + k0 * 2;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(p.rsrc, (lds_void_ptr)(lds_operand + (wave * kGlds + i) * 8 * TK), 16,
                                           chunk_off(p, k0, i & 1, kt), soff, 0, 0);
}

// One K-tile of the kAsmMfma|kInterleave schedule, in 2 x 16 groups fenced by
// sched_barrier(0) so the issue order is exactly this:
//   k-half 0: [4 MFMA(fa0,fb0) + ds_read of one fa1/fb1 fragment] x 16
//   s_waitcnt(0); s_barrier
//   k-half 1: [4 MFMA(fa1,fb1) + one glds of tile t+2 + ds_read of one
//              fa0/fb0 fragment of tile t+1] x 16
// A ds_read overwrites a fragment register >= 16 MFMAs after its last reader
// (WAR on srcA/B of an in-flight MFMA, invisible to the hazard recognizer
// through inline asm).
template <bool INIT, bool EARLY, bool READS_EARLY, bool KT = false, bool NN = false, bool SW = false,
          bool ALT = false, bool STAMP = false, bool NOGLDS = false, bool SPLIT = false, bool SPACED = false,
          bool NOREADS = false, bool CSOFF = false>
__device__ __forceinline__ void ktile_asm(f32x4 (&acc)[8][8], bf16x8 (&fa0)[8], bf16x8 (&fb0)[8], bf16x8 (&fa1)[8],
                                          bf16x8 (&fb1)[8], uint16_t* smem, const Panel& pa, const Panel& pb, int t,
                                          int nk, int wr, int wc, int lane, int wave, StampAcc* sa = nullptr) {
  uint16_t* cur = smem + (t & 1) * kBuf;
  uint16_t* nxt = smem + ((t & 1) ^ 1) * kBuf;
  const int rl = lane & 15, ch = lane >> 4;
  uint64_t tstart = 0;
  if constexpr (STAMP) {
    tstart = __builtin_amdgcn_s_memtime();
    if (sa->t_end) sa->h1 += tstart - sa->t_end;  // the previous K-tile's second half ends here
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    auto mfmas = [&]() {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) mfma_ab<INIT, SW>(acc[g >> 1][(g & 1) * 4 + jj], fa0[g >> 1], fb0[(g & 1) * 4 + jj]);
    };
    auto read1 = [&](int i) {  // i-th of the 16 k-half-1 fragments: fa1[0..7], fb1[0..7]
      if constexpr (NOREADS) return;
      if (i < 8) fa1[i] = frag(cur, wr * 128 + i * 16 + rl, 4 + ch);
      else fb1[i - 8] = fragB(cur + kOperand, wc, i - 8, 1, lane, NN, SW);
    };
    if constexpr (SPACED && !READS_EARLY) {
      mfma_ab<INIT, SW>(acc[g >> 1][(g & 1) * 4 + 0], fa0[g >> 1], fb0[(g & 1) * 4 + 0]);
      mfma_ab<INIT, SW>(acc[g >> 1][(g & 1) * 4 + 1], fa0[g >> 1], fb0[(g & 1) * 4 + 1]);
      __builtin_amdgcn_sched_barrier(0);
      read1(g);
      __builtin_amdgcn_sched_barrier(0);
      mfma_ab<INIT, SW>(acc[g >> 1][(g & 1) * 4 + 2], fa0[g >> 1], fb0[(g & 1) * 4 + 2]);
      mfma_ab<INIT, SW>(acc[g >> 1][(g & 1) * 4 + 3], fa0[g >> 1], fb0[(g & 1) * 4 + 3]);
      __builtin_amdgcn_sched_barrier(0);
      continue;
    }
    if constexpr (!ALT) mfmas();
    if constexpr (READS_EARLY) {
      // all 16 reads by group 11 (2 per group in 0..3): the lgkmcnt(0) before
      // the barrier then has 16 MFMAs to cover the last read's latency
      if (g < 4) {
        read1(2 * g);
        read1(2 * g + 1);
      } else if (g < 12) {
        read1(g + 4);
      }
    } else {
      read1(g);
    }
    if constexpr (ALT) {
      __builtin_amdgcn_sched_barrier(0);
      mfmas();
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  uint64_t ts0 = 0;
  if constexpr (STAMP) ts0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  barrier();
  if constexpr (STAMP) {
    const uint64_t ts1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sa->wait += ts1 - ts0;
    sa->h0 += ts0 - tstart;
    sa->t_end = ts1;
  }
  const int kn = min(t + 2, nk - 1) * TK;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    auto mfmas = [&]() {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) mfma_ab<false, SW>(acc[g >> 1][(g & 1) * 4 + jj], fa1[g >> 1], fb1[(g & 1) * 4 + jj]);
    };
    if constexpr (SPACED && !EARLY && !NOGLDS && !SPLIT) {
      auto m1 = [&](int jj) { mfma_ab<false, SW>(acc[g >> 1][(g & 1) * 4 + jj], fa1[g >> 1], fb1[(g & 1) * 4 + jj]); };
      m1(0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (CSOFF && !NN && !KT) {
        // descriptor moved to column kn; the row offsets are loop-invariant
        const Panel& p = g < 8 ? pa : pb;
        const int i = g & 7;
        const uint64_t base = (((uint64_t)p.w.y) << 32 | p.w.x) + (uint64_t)kn * 2;
        srd4 w = p.w;
        w.x = (uint32_t)base;
        w.y = (uint32_t)(base >> 32);
        w.z = p.w.z - (uint32_t)(kn * 2);
        glds_raw(w, (g < 8 ? cur : cur + kOperand) + (wave * kGlds + i) * 8 * TK, p.lane_off[i & 1],
                 (wave * 64 + i * 8) * p.row_bytes);
      } else if (g < 8) {
        if constexpr (NN) glds_a_raw(pa, kn, cur, wave, g);
        else glds_one(pa, kn, cur, wave, g, KT);
      } else if constexpr (NN) {
        glds_nn(pb, kn, cur + kOperand, wave, g - 8);
      } else {
        glds_one(pb, kn, cur + kOperand, wave, g - 8, KT);
      }
      __builtin_amdgcn_sched_barrier(0);
      m1(1);
      m1(2);
      __builtin_amdgcn_sched_barrier(0);
      if (g == 0) fa0[0] = frag(nxt, wr * 128 + rl, ch);
      else if (g <= 8) fb0[g - 1] = fragB(nxt + kOperand, wc, g - 1, 0, lane, NN, SW);
      else fa0[g - 8] = frag(nxt, wr * 128 + (g - 8) * 16 + rl, ch);
      __builtin_amdgcn_sched_barrier(0);
      m1(3);
      __builtin_amdgcn_sched_barrier(0);
      continue;
    }
    if constexpr (!ALT) mfmas();
    if constexpr (NOGLDS) {
    } else if constexpr (EARLY || SPLIT) {  // all 16 glds in the first 8 groups: more time to land
      if (g < 8) {
        if constexpr (NN) glds_a_raw(pa, kn, cur, wave, g);
        else glds_one(pa, kn, cur, wave, g, KT);
        if constexpr (NN) glds_nn(pb, kn, cur + kOperand, wave, g);
        else glds_one(pb, kn, cur + kOperand, wave, g, KT);
      }
    } else {
      if (g < 8) {
        if constexpr (NN) glds_a_raw(pa, kn, cur, wave, g);
        else glds_one(pa, kn, cur, wave, g, KT);
      }
      else if constexpr (NN) glds_nn(pb, kn, cur + kOperand, wave, g - 8);
      else glds_one(pb, kn, cur + kOperand, wave, g - 8, KT);
    }
    // in the order the next K-tile's first groups consume them: fa0[0],
    // fb0[0..7], fa0[1..7]
    auto read0 = [&](int i) {
      if constexpr (NOREADS) return;
      if (i == 0) fa0[0] = frag(nxt, wr * 128 + rl, ch);
      else if (i <= 8) fb0[i - 1] = fragB(nxt + kOperand, wc, i - 1, 0, lane, NN, SW);
      else fa0[i - 8] = frag(nxt, wr * 128 + (i - 8) * 16 + rl, ch);
    };
    if constexpr (SPLIT) {
      if (g >= 8) {
        read0(2 * (g - 8));
        read0(2 * (g - 8) + 1);
      }
    } else {
      read0(g);
    }
    if constexpr (ALT) {
      __builtin_amdgcn_sched_barrier(0);
      mfmas();
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// the i-th glds of one operand's K-tile as inline asm (glds_one's addressing):
// invisible to the compiler's LDS-DMA alias tracking, so no vmcnt wait lands
// before the ds_reads of the other operand's region that run beside it
template <bool NN_B>
__device__ __forceinline__ void glds_any_raw(const Panel& p, int k0, uint16_t* lds_operand, int wave, int i,
                                             bool kt) {
  if constexpr (NN_B) {
    glds_nn(p, k0, lds_operand, wave, i);
  } else {
    const int soff = (wave * 64 + i * 8) * p.row_bytes + k0 * 2;
    glds_raw(p.w, lds_operand + (wave * kGlds + i) * 8 * TK, chunk_off(p, k0, i & 1, kt), soff);
  }
}

// One K-tile with three barriers (kThreeBar), 32 groups of 4 MFMAs fenced by
// sched_barrier(0); group g runs k-half g >> 4:
//   g 0-3    ds_read fa1[0..7] (2 per group)                      [cur A]
//   g 5      s_waitcnt lgkmcnt(0); s_barrier   -> cur's A region free
//   g 6-11   glds A of tile t+2 -> cur (2,2,1,1,1,1); ds_read fb1 (g 6-9, 2 each)
//   g 11     s_waitcnt lgkmcnt(0); s_barrier   -> cur's B region free
//   g 12-19  glds B of tile t+2 -> cur (1 per group)
//   g 22     s_waitcnt vmcnt(16); s_barrier    -> tile t+1 (issued one
//            iteration earlier) landed for every wave
//   g 23-30  ds_read fa0/fb0 of tile t+1 (2 per group)             [nxt]
// A K-tile load now has from its issue (MFMA 24-80) to MFMA 92 of the next
// iteration to land (~100-200 MFMAs, vs 64-128 in ktile_asm), the shape of
// the schedule hipBLASLt's MT256x256x64 kernel runs on gfx950
// (Custom_Cijk_Alik_Bljk_..._MT256x256x64_MI16x16x1, its main loop read off a
// static disassembly of the library's code object).  WAR: a fragment register
// is overwritten >= 12 MFMAs after its last reader.
template <bool INIT, bool KT = false, bool NN = false, bool SPREAD = false>
__device__ __forceinline__ void ktile_asm3(f32x4 (&acc)[8][8], bf16x8 (&fa0)[8], bf16x8 (&fb0)[8], bf16x8 (&fa1)[8],
                                           bf16x8 (&fb1)[8], uint16_t* smem, const Panel& pa, const Panel& pb, int t,
                                           int nk, int wr, int wc, int lane, int wave) {
  uint16_t* cur = smem + (t & 1) * kBuf;
  uint16_t* nxt = smem + ((t & 1) ^ 1) * kBuf;
  const int rl = lane & 15, ch = lane >> 4;
  const int kn = min(t + 2, nk - 1) * TK;
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int g = 0; g < 32; ++g) {
    const int h = g & 15;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      if (g < 16) mfma_asm<INIT>(acc[h >> 1][(h & 1) * 4 + jj], fa0[h >> 1], fb0[(h & 1) * 4 + jj]);
      else mfma_asm<false>(acc[h >> 1][(h & 1) * 4 + jj], fa1[h >> 1], fb1[(h & 1) * 4 + jj]);
    }
    if (g < 4) {
      fa1[2 * g] = frag(cur, wr * 128 + 2 * g * 16 + rl, 4 + ch);
      fa1[2 * g + 1] = frag(cur, wr * 128 + (2 * g + 1) * 16 + rl, 4 + ch);
    }
    if constexpr (SPREAD) {
      // one glds every other group: A at g = 6, 8, .., 20, B at g = 12, .., 26
      if (g >= 6 && g <= 20 && (g & 1) == 0) {
        if constexpr (NN) glds_a_raw(pa, kn, cur, wave, (g - 6) >> 1);
        else glds_any_raw<false>(pa, kn, cur, wave, (g - 6) >> 1, KT);
      }
      if (g >= 12 && g <= 26 && (g & 1) == 0) glds_any_raw<NN>(pb, kn, cur + kOperand, wave, (g - 12) >> 1, KT);
    } else if (g >= 6 && g < 12) {
      const int i0 = g < 8 ? 2 * (g - 6) : g - 4;  // A glds 0,1 | 2,3 | 4 | 5 | 6 | 7
      const int n = g < 8 ? 2 : 1;
      for (int q = 0; q < n; ++q) {
        if constexpr (NN) glds_a_raw(pa, kn, cur, wave, i0 + q);
        else glds_any_raw<false>(pa, kn, cur, wave, i0 + q, KT);
      }
    }
    if (g >= 6 && g < 10) {
      fb1[2 * (g - 6)] = fragB(cur + kOperand, wc, 2 * (g - 6), 1, lane, NN);
      fb1[2 * (g - 6) + 1] = fragB(cur + kOperand, wc, 2 * (g - 6) + 1, 1, lane, NN);
    }
    if (!SPREAD && g >= 12 && g < 20) glds_any_raw<NN>(pb, kn, cur + kOperand, wave, g - 12, KT);
    if (g >= 23 && g < 31) {
      // in the order the next K-tile's first groups consume them: fa0[0],
      // fb0[0..7], fa0[1..7]
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = 2 * (g - 23) + q;
        if (i == 0) fa0[0] = frag(nxt, wr * 128 + rl, ch);
        else if (i <= 8) fb0[i - 1] = fragB(nxt + kOperand, wc, i - 1, 0, lane, NN);
        else fa0[i - 8] = frag(nxt, wr * 128 + (i - 8) * 16 + rl, ch);
      }
    }
    if (g == 5 || g == 11) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier();
    } else if (g == 22) {
      // tile t+1 landed: all but the glds of tile t+2 issued so far retired
      if constexpr (SPREAD) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      barrier();
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One K-tile with two barriers (kTwoBar): the K-tile wait moves from the
// k-half boundary to the middle of the second k-half.  32 groups of 4 MFMAs
// fenced by sched_barrier(0), as ktile_asm's kSpacedMem form:
//   k-half 0, g 0-7    2 ds_read of the k-half-1 fragments (cur) per group,
//                      between the MFMA pairs: all 16 issued by MFMA 32, so
//                      the lgkmcnt(0) below has 32 MFMAs to cover them
//   end of k-half 0    s_waitcnt lgkmcnt(0); s_barrier   -> cur is free
//   k-half 1, g 0-7    one glds of tile t+2 -> cur per group (A)
//   k-half 1, g 8      s_waitcnt vmcnt(8); s_barrier     -> tile t+1 (the glds
//                      one iteration earlier) landed for every wave; only this
//                      iteration's 8 younger glds may still be in flight
//   k-half 1, g 8-15   one glds (B) + 2 ds_read of tile t+1's k-half-0
//                      fragments (nxt) per group, in the order the next
//                      K-tile consumes them
// Why: PMC at 8192^3 (profiles/r4_gemm_pmc.md) put the gap to hipBLASLt in
// SQ_WAIT_ANY -- 423 vs 105 cycles per wave per K-tile at equal
// SQ_WAIT_INST_ANY -- and the one-barrier loop gave a K-tile load only
// 68-128 MFMAs to land; here it has 100-160.  WAR: the earliest k-half-1
// fragment write lands >= 20 MFMAs after its last reader (fa1[i] first, then
// fb1[0..3], fa1[6], fb1[4..7], fa1[7]: each after its last use + 16).
template <bool INIT, bool KT = false, bool NN = false, int WG = 8, int DIAG = 0, bool SW = false, int RG = 8>
__device__ __forceinline__ void ktile_asm2(f32x4 (&acc)[8][8], bf16x8 (&fa0)[8], bf16x8 (&fb0)[8], bf16x8 (&fa1)[8],
                                           bf16x8 (&fb1)[8], uint16_t* smem, const Panel& pa, const Panel& pb, int t,
                                           int nk, int wr, int wc, int lane, int wave) {
  uint16_t* cur = smem + (t & 1) * kBuf;
  uint16_t* nxt = smem + ((t & 1) ^ 1) * kBuf;
  const int rl = lane & 15, ch = lane >> 4;
  // k-half-1 fragment j of the 16 in WAR-safe order (see above): 0-5 fa1[0..5],
  // 6-9 fb1[0..3], 10 fa1[6], 11-14 fb1[4..7], 15 fa1[7]
  auto read1 = [&](int j) {
    if (j < 6) fa1[j] = frag(cur, wr * 128 + j * 16 + rl, 4 + ch);
    else if (j < 10) fb1[j - 6] = fragB(cur + kOperand, wc, j - 6, 1, lane, NN, SW);
    else if (j == 10) fa1[6] = frag(cur, wr * 128 + 6 * 16 + rl, 4 + ch);
    else if (j < 15) fb1[j - 7] = fragB(cur + kOperand, wc, j - 7, 1, lane, NN, SW);
    else fa1[7] = frag(cur, wr * 128 + 7 * 16 + rl, 4 + ch);
  };
  // tile t+1's k-half-0 fragment i, in consumption order: fa0[0], fb0[0..7], fa0[1..7]
  auto read0 = [&](int i) {
    if (i == 0) fa0[0] = frag(nxt, wr * 128 + rl, ch);
    else if (i <= 8) fb0[i - 1] = fragB(nxt + kOperand, wc, i - 1, 0, lane, NN, SW);
    else fa0[i - 8] = frag(nxt, wr * 128 + (i - 8) * 16 + rl, ch);
  };
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    auto m0 = [&](int jj) { mfma_ab<INIT, SW>(acc[g >> 1][(g & 1) * 4 + jj], fa0[g >> 1], fb0[(g & 1) * 4 + jj]); };
    // RG = 8: reads 2g, 2g+1 in group g < 8; RG = 12: reads 2g, 2g+1 in
    // groups 0-3, read g + 4 in groups 4-11 (the same order, so the same WAR
    // distances or longer)
    constexpr bool two = RG == 8 ? true : false;
    m0(0);
    __builtin_amdgcn_sched_barrier(0);
    if (two ? g < 8 : g < 4) read1(2 * g);
    else if (!two && g < 12) read1(g + 4);
    __builtin_amdgcn_sched_barrier(0);
    m0(1);
    __builtin_amdgcn_sched_barrier(0);
    if (two ? g < 8 : g < 4) read1(2 * g + 1);
    __builtin_amdgcn_sched_barrier(0);
    m0(2);
    m0(3);
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr ((DIAG & kDiagNoBar1) == 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
  }
  const int kn = min(t + 2, nk - 1) * TK;
  static_assert(WG == 8 || WG == 10 || WG == 12, "kTwoBar wait group");
  // tile t+1's 16 fragment reads over groups WG..15: read i in group
  // WG + i * (16 - WG) / 16, up to 4 per group, one after each of MFMA 1-3
  // (and a 4th after the last)
  constexpr int kSpan = 16 - WG;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    auto m1 = [&](int jj) { mfma_ab<false, SW>(acc[g >> 1][(g & 1) * 4 + jj], fa1[g >> 1], fb1[(g & 1) * 4 + jj]); };
    if (g == WG) {
      // tile t+1 landed: only this iteration's WG younger glds may be in flight
      if constexpr ((DIAG & kDiagNoVmWait) != 0) {
      } else if constexpr (WG == 8) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else if constexpr (WG == 10) {
        asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      }
      if constexpr ((DIAG & kDiagNoBar2) == 0) barrier();
    }
    m1(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((DIAG & kDiagNoGlds) != 0) {
    } else if (g < 8) {
      if constexpr (NN) glds_a_raw(pa, kn, cur, wave, g);
      else glds_one(pa, kn, cur, wave, g, KT);
    } else if constexpr (NN) {
      glds_nn(pb, kn, cur + kOperand, wave, g - 8);
    } else {
      glds_one(pb, kn, cur + kOperand, wave, g - 8, KT);
    }
    __builtin_amdgcn_sched_barrier(0);
    // the reads of this group: i with WG + i * kSpan / 16 == g
    int k = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (g >= WG && WG + i * kSpan / 16 == g) {
        if (k < 3) m1(1 + k);  // (a 4th read of the group follows the 4th MFMA)
        __builtin_amdgcn_sched_barrier(0);
        if constexpr ((DIAG & kDiagNoReads0) == 0) read0(i);
        __builtin_amdgcn_sched_barrier(0);
        ++k;
      }
    }
#pragma unroll
    for (int jj = 1; jj < 4; ++jj)
      if (jj > k) m1(jj);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <bool OUT_BF16, bool NT = false>
__device__ __forceinline__ void epilogue(uint16_t* smem, const f32x4 (&acc)[8][8], void* __restrict__ C, int ldc,
                                         int64_t row0, int col0, int wave, int lane, float alpha, float beta) {
  float* ep = reinterpret_cast<float*>(smem) + wave * kEpWaveFloats;
#pragma unroll
  for (int half = 0; half < 4; ++half) {  // 32 output rows (2 fragment rows) per round
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ep[(ii * 16 + (lane >> 4) * 4 + r) * kEpPitch + j * 16 + (lane & 15)] = alpha * acc[half * 2 + ii][j][r];
    const int64_t grow0 = row0 + half * 32;
    if constexpr (OUT_BF16) {
      // 16 lanes x 8 columns per row, 4 rows per pass
#pragma unroll
      for (int it = 0; it < kEpRows / 4; ++it) {
        const int row = it * 4 + (lane >> 4), col = (lane & 15) * 8;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(ep + row * kEpPitch + col);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(ep + row * kEpPitch + col + 4);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        uint4* dst = reinterpret_cast<uint4*>((uint16_t*)C + (grow0 + row) * ldc + col0 + col);
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
        if constexpr (NT) {
          typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
          const u32x4 pk = {packed[0], packed[1], packed[2], packed[3]};
          __builtin_nontemporal_store(pk, reinterpret_cast<u32x4*>(dst));
        } else {
          *dst = make_uint4(packed[0], packed[1], packed[2], packed[3]);
        }
      }
    } else {
      // 32 lanes x 4 columns per row, 2 rows per pass
#pragma unroll
      for (int it = 0; it < kEpRows / 2; ++it) {
        const int row = it * 2 + (lane >> 5), col = (lane & 31) * 4;
        f32x4 v = *reinterpret_cast<const f32x4*>(ep + row * kEpPitch + col);
        f32x4* dst = reinterpret_cast<f32x4*>((float*)C + (grow0 + row) * ldc + col0 + col);
        if (beta != 0.f) v += beta * *dst;
        if constexpr (NT) __builtin_nontemporal_store(v, dst);
        else *dst = v;
      }
    }
  }
}

// kSwapAB epilogue: lane (g = lane >> 4) holds row wr*128 + 16i + (lane & 15),
// columns 32p + 8g + 0..7 in acc[i][2p] (first 4) and acc[i][2p+1] (last 4):
// one 16-B store per (i, p) for bf16 C, two for f32 C.  MASKED: the ragged
// border, element by element.
template <bool OUT_BF16, bool MASKED>
__device__ __forceinline__ void epilogue_rows(const f32x4 (&acc)[8][8], void* __restrict__ C, int ldc, int64_t row0,
                                              int col0, int M, int N, int lane, float alpha, float beta) {
  const int g = lane >> 4, rl = lane & 15;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t row = row0 + i * 16 + rl;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int col = col0 + 32 * p + 8 * g;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = alpha * acc[i][2 * p][e];
        v[4 + e] = alpha * acc[i][2 * p + 1][e];
      }
      if constexpr (MASKED) {
        if (row >= M) continue;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (col + e >= N) break;
          if constexpr (OUT_BF16) {
            uint16_t* dst = (uint16_t*)C + row * ldc + col + e;
            float x = v[e];
            if (beta != 0.f) x += beta * bf16_bits_to_float(*dst);
            *dst = float_to_bf16_bits(x);
          } else {
            float* dst = (float*)C + row * ldc + col + e;
            *dst = v[e] + (beta != 0.f ? beta * *dst : 0.f);
          }
        }
      } else if constexpr (OUT_BF16) {
        uint4* dst = reinterpret_cast<uint4*>((uint16_t*)C + row * ldc + col);
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
        typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
        const u32x4 pk = {packed[0], packed[1], packed[2], packed[3]};
        __builtin_nontemporal_store(pk, reinterpret_cast<u32x4*>(dst));
      } else {
        f32x4* dst = reinterpret_cast<f32x4*>((float*)C + row * ldc + col);
        f32x4 lo = {v[0], v[1], v[2], v[3]}, hi = {v[4], v[5], v[6], v[7]};
        if (beta != 0.f) {
          lo += beta * dst[0];
          hi += beta * dst[1];
        }
        __builtin_nontemporal_store(lo, dst);
        __builtin_nontemporal_store(hi, dst + 1);
      }
    }
  }
}

// kEdge border blocks: the same LDS staging, element stores under the
// (row < M, col < N) mask; no alignment assumed of C or ldc
template <bool OUT_BF16>
__device__ __forceinline__ void epilogue_masked(uint16_t* smem, const f32x4 (&acc)[8][8], void* __restrict__ C,
                                                int ldc, int64_t row0, int col0, int M, int N, int wave, int lane,
                                                float alpha, float beta) {
  float* ep = reinterpret_cast<float*>(smem) + wave * kEpWaveFloats;
#pragma unroll
  for (int half = 0; half < 4; ++half) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ep[(ii * 16 + (lane >> 4) * 4 + r) * kEpPitch + j * 16 + (lane & 15)] = alpha * acc[half * 2 + ii][j][r];
    const int64_t grow0 = row0 + half * 32;
    // 64 lanes x 2 columns per row, one row per pass: consecutive lanes,
    // consecutive addresses
#pragma unroll 4
    for (int row = 0; row < kEpRows; ++row) {
      const int64_t grow = grow0 + row;
      if (grow >= M) break;  // wave-uniform
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int col = e * 64 + lane;
        const int gcol = col0 + col;
        if (gcol >= N) continue;
        float v = ep[row * kEpPitch + col];
        if constexpr (OUT_BF16) {
          uint16_t* dst = (uint16_t*)C + grow * ldc + gcol;
          if (beta != 0.f) v += beta * bf16_bits_to_float(*dst);
          *dst = float_to_bf16_bits(v);
        } else {
          float* dst = (float*)C + grow * ldc + gcol;
          if (beta != 0.f) v += beta * *dst;
          *dst = v;
        }
      }
    }
  }
}

template <bool OUT_BF16, long long O>
__global__ __launch_bounds__(kThreads, 1) void gemm_bf16_tn_256w4(const uint16_t* __restrict__ A,
                                                                  const uint16_t* __restrict__ Bt,
                                                                  void* __restrict__ C, int M, int N, int K, int lda,
                                                                  int ldb, int ldc, float alpha, float beta) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[kSmemBytes / 2];  // the only LDS object
  constexpr bool pin = (O & kPinOrder) != 0, inter = (O & kInterleave) != 0, am = (O & kAsmMfma) != 0,
                 early = (O & kEarlyGlds) != 0, reads_early = (O & kReadsEarly) != 0;

  constexpr bool edge = (O & kEdge) != 0, nn = (O & kNN) != 0, sw = (O & kSwapAB) != 0;
  static_assert(!(edge && nn), "kNN is for tile-multiple shapes");
  static_assert(!(sw && nn), "kSwapAB permutes B's rows: TN only");
  static_assert(!sw || (am && inter && (O & kThreeBar) == 0), "kSwapAB: the ktile_asm / ktile_asm2 schedules");
  const int nbm = edge ? (M + TM - 1) / TM : M / TM, nbn = edge ? (N + TN - 1) / TN : N / TN, nblocks = nbm * nbn;
  const int b = xcd_remap(blockIdx.x, nblocks);
  constexpr int kGm = (O & kGroup2) ? 2 : (O & kGroup8) ? 8 : (O & kGroup16) ? 16 : kGroupM;
  const int group = kGm * nbn;
  const int first_m = (b / group) * kGm;
  const int gm = min(nbm - first_m, kGm);
  const int tm = first_m + (b % group) % gm, tn = (b % group) / gm;
  const int m0 = tm * TM, n0 = tn * TN;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  Panel pa = make_panel(A + (int64_t)m0 * lda, lda, lane, edge ? min(TM, M - m0) : TM, K);
  if constexpr (nn) {
    const int64_t span = (int64_t)TM * lda * 2;
    pa.w = srd_words(A + (int64_t)m0 * lda, span > 0xffffffffll ? 0xffffffffu : (uint32_t)span);
  }
  const Panel pb = nn ? make_panel_nn(Bt + n0, ldb, lane, K)
                      : make_panel(Bt + (int64_t)n0 * ldb, ldb, lane, edge ? min(TN, N - n0) : TN, K);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = edge ? (K + TK - 1) / TK : K / TK;  // kEdge: a ragged last K-tile reads zeros past K
  // prologue: tiles 0 and 1 in flight, wait for tile 0 (16 glds per tile)
  stage(pa, 0, smem, wave, edge, false, nn);
  stage(pb, 0, smem + kOperand, wave, edge, nn);
  if (nk > 1) {
    stage(pa, TK, smem + kBuf, wave, edge, false, nn);
    stage(pb, TK, smem + kBuf + kOperand, wave, edge, nn);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();

  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  if constexpr (am && inter && (O & kThreeBar) != 0) {
    read_frags(smem, wr, wc, lane, 0, fa0, fb0, nn);
    constexpr bool spread = (O & kSpread) != 0;
    ktile_asm3<true, edge, nn, spread>(acc, fa0, fb0, fa1, fb1, smem, pa, pb, 0, nk, wr, wc, lane, wave);
    for (int t = 1; t < nk; ++t)
      ktile_asm3<false, edge, nn, spread>(acc, fa0, fb0, fa1, fb1, smem, pa, pb, t, nk, wr, wc, lane, wave);
  } else if constexpr (am && inter && (O & kTwoBar) != 0) {
    constexpr int wg = (O & kTwoBarG10) ? 10 : (O & kTwoBarG12) ? 12 : 8;
    constexpr int diag = (int)(O & (kDiagNoVmWait | kDiagNoBar2 | kDiagNoBar1 | kDiagNoReads0 | kDiagNoGlds));
    constexpr int rg = (O & kReads12) ? 12 : 8;
    read_frags(smem, wr, wc, lane, 0, fa0, fb0, nn, sw);
    ktile_asm2<true, edge, nn, wg, diag, sw, rg>(acc, fa0, fb0, fa1, fb1, smem, pa, pb, 0, nk, wr, wc, lane, wave);
    for (int t = 1; t < nk; ++t)
      ktile_asm2<false, edge, nn, wg, diag, sw, rg>(acc, fa0, fb0, fa1, fb1, smem, pa, pb, t, nk, wr, wc, lane, wave);
  } else if constexpr (am && inter && (O & kAltSimd) != 0) {
    read_frags(smem, wr, wc, lane, 0, fa0, fb0, nn, sw);
    // HW_ID bit 4 = the SIMD's parity (s_getreg_b32 hwreg(HW_REG_HW_ID, 4, 1))
    if (__builtin_amdgcn_s_getreg((0 << 11) | (4 << 6) | 4) & 1) {
      ktile_asm<true, early, reads_early, edge, nn, sw, true>(acc, fa0, fb0, fa1, fb1, smem, pa, pb, 0, nk, wr, wc, lane, wave);
      for (int t = 1; t < nk; ++t)
        ktile_asm<false, early, reads_early, edge, nn, sw, true>(acc, fa0, fb0, fa1, fb1, smem, pa, pb, t, nk, wr, wc, lane, wave);
    } else {
      ktile_asm<true, early, reads_early, edge, nn, sw>(acc, fa0, fb0, fa1, fb1, smem, pa, pb, 0, nk, wr, wc, lane, wave);
      for (int t = 1; t < nk; ++t)
        ktile_asm<false, early, reads_early, edge, nn, sw>(acc, fa0, fb0, fa1, fb1, smem, pa, pb, t, nk, wr, wc, lane, wave);
    }
  } else if constexpr (am && inter && (O & kDiagStamps) != 0) {
    StampAcc sa;
    read_frags(smem, wr, wc, lane, 0, fa0, fb0, nn, sw);
    const uint64_t tl0 = __builtin_amdgcn_s_memtime();
    constexpr bool nor = (O & kDiagMfmaOnly) != 0, cso = (O & kConstSoff) != 0;
    constexpr bool nog = (O & kDiagNoGlds) != 0 || nor, spl = (O & kSplitGlds) != 0, spc = (O & kSpacedMem) != 0;
    if constexpr (nor) read_frags(smem, wr, wc, lane, 1, fa1, fb1, nn, sw);
    ktile_asm<true, early, reads_early, edge, nn, sw, false, true, nog, spl, spc, nor, cso>(
        acc, fa0, fb0, fa1, fb1, smem, pa, pb, 0, nk, wr, wc, lane, wave, &sa);
    for (int t = 1; t < nk; ++t)
      ktile_asm<false, early, reads_early, edge, nn, sw, false, true, nog, spl, spc, nor, cso>(
          acc, fa0, fb0, fa1, fb1, smem, pa, pb, t, nk, wr, wc, lane, wave, &sa);
    const uint64_t tl1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    barrier();
    if constexpr (am) mfma_drain();
    // the accumulators must stay live (the MFMAs are not volatile): fold
    // them into one value nobody reads back as data
    float keep = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) keep += acc[i][j][0] + acc[i][j][3];
    if (lane == 0) {
      uint32_t* st = reinterpret_cast<uint32_t*>((char*)C + 16 * ((size_t)blockIdx.x * 4 + wave));
      st[0] = (uint32_t)(tl1 - tl0);
      st[1] = (uint32_t)sa.wait;
      st[2] = (uint32_t)sa.h0 | ((uint32_t)nk << 24);  // h0 < 2^24 cycles at these sizes; nk < 256
      st[3] = (uint32_t)(sa.h1 + (tl1 - sa.t_end)) ^ (__float_as_uint(keep) & 1u);  // (the last half-1 ends at tl1)
    }
    return;
  } else if constexpr (am && inter) {
    // hand-interleaved pipeline; K-tile 0 peeled so its MFMAs start the
    // accumulators from the constant 0 (no AGPR zero-fill to fence)
    constexpr bool nog = (O & kDiagNoGlds) != 0, spl = (O & kSplitGlds) != 0, spc = (O & kSpacedMem) != 0,
                   cso = (O & kConstSoff) != 0;
    read_frags(smem, wr, wc, lane, 0, fa0, fb0, nn, sw);
    ktile_asm<true, early, reads_early, edge, nn, sw, false, false, nog, spl, spc, false, cso>(
        acc, fa0, fb0, fa1, fb1, smem, pa, pb, 0, nk, wr, wc, lane, wave);
    for (int t = 1; t < nk; ++t)
      ktile_asm<false, early, reads_early, edge, nn, sw, false, false, nog, spl, spc, false, cso>(
          acc, fa0, fb0, fa1, fb1, smem, pa, pb, t, nk, wr, wc, lane, wave);
  } else if constexpr ((O & kNoCarry) != 0) {
    // loop-carried state is the accumulators only (simpler register
    // allocation); the first MFMAs of each K-tile wait for its first reads
    for (int t = 0; t < nk; ++t) {
      uint16_t* cur = smem + (t & 1) * kBuf;
      read_frags(cur, wr, wc, lane, 0, fa0, fb0, nn);
      read_frags(cur, wr, wc, lane, 1, fa1, fb1, nn);
      mfma_block<am>(acc, fa0, fb0);
      mfma_block<am>(acc, fa1, fb1);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      barrier();
      const int kn = min(t + 2, nk - 1) * TK;
      stage(pa, kn, cur, wave, edge, false, nn);
      stage(pb, kn, cur + kOperand, wave, edge, nn);
    }
  } else {
  read_frags(smem, wr, wc, lane, 0, fa0, fb0, nn);
  for (int t = 0; t < nk; ++t) {
    uint16_t* cur = smem + (t & 1) * kBuf;
    uint16_t* nxt = smem + ((t & 1) ^ 1) * kBuf;

    read_frags(cur, wr, wc, lane, 1, fa1, fb1, nn);
    if constexpr (inter) interleave_hint<16, 0>();
    else if constexpr (pin) __builtin_amdgcn_sched_barrier(0);
    mfma_block<am>(acc, fa0, fb0);
    if constexpr (pin || inter) __builtin_amdgcn_sched_barrier(0);

    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    barrier();

    // branch-free so the loads can be spread among the MFMAs below: past
    // the end, re-stage the last K-tile into the buffer nobody reads again
    // and read fragments nobody uses
    const int kn = min(t + 2, nk - 1) * TK;
    stage(pa, kn, cur, wave, edge, false, nn);
    stage(pb, kn, cur + kOperand, wave, edge, nn);
    read_frags(nxt, wr, wc, lane, 0, fa0, fb0, nn);
    if constexpr (inter) interleave_hint<16, 16>();
    else if constexpr (pin) __builtin_amdgcn_sched_barrier(0);
    mfma_block<am>(acc, fa1, fb1);
    if constexpr (pin || inter) __builtin_amdgcn_sched_barrier(0);
  }
  }

  // every wave's last LDS reads and tail glds retired before any wave's
  // staging writes
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  barrier();
  if constexpr (am) mfma_drain();
  if constexpr ((O & kDiagNoEpilogue) != 0) {
    if (blockIdx.x != 0) return;
  }
  if constexpr (sw) {
    // no LDS staging: the loop's trailing barrier above is all the epilogue needs
    const bool ragged = edge && (m0 + TM > M || n0 + TN > N || (ldc % (OUT_BF16 ? 8 : 4)) != 0 || ((uintptr_t)C & 15) != 0);
    if (ragged)
      epilogue_rows<OUT_BF16, true>(acc, C, ldc, m0 + wr * 128, n0 + wc * 128, M, N, lane, alpha, beta);
    else
      epilogue_rows<OUT_BF16, false>(acc, C, ldc, m0 + wr * 128, n0 + wc * 128, M, N, lane, alpha, beta);
  } else if constexpr ((O & kDirectStore) != 0) {
    // 16x16 C/D map: lane holds rows 4*(lane/16)+r of column lane%16 -> 4
    // scattered element stores per fragment (f32 output only; cheap on
    // registers, expensive on store issue)
    const int64_t r0 = m0 + wr * 128, c0 = n0 + wc * 128;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = r0 + i * 16 + (lane >> 4) * 4 + r;
          const int col = c0 + j * 16 + (lane & 15);
          if constexpr (OUT_BF16) ((uint16_t*)C)[row * ldc + col] = float_to_bf16_bits(alpha * acc[i][j][r]);
          else ((float*)C)[row * ldc + col] = alpha * acc[i][j][r] + (beta != 0.f ? beta * ((float*)C)[row * ldc + col] : 0.f);
        }
  } else if (edge && (m0 + TM > M || n0 + TN > N || (ldc % (OUT_BF16 ? 8 : 4)) != 0 ||
                      ((uintptr_t)C & 15) != 0)) {
    epilogue_masked<OUT_BF16>(smem, acc, C, ldc, m0 + wr * 128, n0 + wc * 128, M, N, wave, lane, alpha, beta);
  } else {
    epilogue<OUT_BF16, (O & kNtStore) != 0>(smem, acc, C, ldc, m0 + wr * 128, n0 + wc * 128, wave, lane, alpha, beta);
  }
}

inline bool ok(int M, int N, int K, int lda, int ldb, int ldc, bool out_bf16) {
  // a panel's loads use 32-bit buffer offsets ((wave*64 + i*8) * ld*2 + k0*2
  // in an SGPR, a 256-row extent in the descriptor): leading dimensions whose
  // 256-row span does not fit 31 bits go to the 8-wave kernel (64-bit math)
  const auto span_ok = [K](int ld) { return (int64_t)256 * ld * 2 + (int64_t)K * 2 < 0x7fffffffll; };
  return M > 0 && N > 0 && K > 0 && M % TM == 0 && N % TN == 0 && K % TK == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldc % (out_bf16 ? 8 : 4) == 0 && span_ok(lda) && span_ok(ldb);
}

// kNN: B is [K][N]; tile multiples; the K x ldb panel within 31-bit offsets
inline bool nn_ok(int M, int N, int K, int lda, int ldb, int ldc, bool out_bf16) {
  const auto span_ok = [K](int ld) { return (int64_t)256 * ld * 2 + (int64_t)K * 2 < 0x7fffffffll; };
  return M > 0 && N > 0 && K > 0 && M % TM == 0 && N % TN == 0 && K % TK == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldb >= N && ldc % (out_bf16 ? 8 : 4) == 0 && span_ok(lda) && (int64_t)K * ldb * 2 < 0x7fffffffll;
}

// kEdge: any M, N; the rest as ok()
inline bool edge_ok(int M, int N, int K, int lda, int ldb) {
  const auto span_ok = [K](int ld) { return (int64_t)256 * ld * 2 + (int64_t)K * 2 < 0x7fffffffll; };
  return M > 0 && N > 0 && K > 0 && K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && span_ok(lda) && span_ok(ldb);
}

template <long long O>
inline void launch(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
                   float beta, bool out_bf16, hipStream_t stream) {
  const unsigned grid = (O & kEdge) ? (unsigned)(((M + TM - 1) / TM) * ((N + TN - 1) / TN))
                                    : (unsigned)((M / TM) * (N / TN));
  if (out_bf16)
    gemm_bf16_tn_256w4<true, O><<<grid, kThreads, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K,
                                                               lda, ldb, ldc, alpha, beta);
  else
    gemm_bf16_tn_256w4<false, O><<<grid, kThreads, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K,
                                                                lda, ldb, ldc, alpha, beta);
}

}  // namespace g4
}  // namespace bk
