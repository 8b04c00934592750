// bf16 GEMM on gfx950 matrix cores: C[M,N] = alpha * A[M,K] . Bt[N,K]^T
// (+ beta * C), f32 accumulation, bf16 or f32 output.
//
// Fast path (M%128 == N%128 == K%64 == 0, 16-B aligned rows): 128x128x64
// block tile, 256 threads = 4 waves in 2x2, each wave a 64x64 sub-tile of
// 4x4 `v_mfma_f32_16x16x32_bf16` accumulators (64 AGPR/VGPR).  Operands go
// HBM -> LDS with `global_load_lds_dwordx4` (one wave-instruction = 1 KiB =
// 8 tile rows; no VGPR staging), two LDS buffers so tile t+1 streams in while
// tile t is multiplied.  The LDS image is lane-linear (a DMA constraint), so
// the bank-conflict XOR swizzle is applied to the per-lane GLOBAL source
// address and undone on the ds_read_b128 address (cdna_hip_programming §5.4
// rule 21): 16-B chunk c of row r lives at chunk c ^ ((r >> 1) & 7), which
// makes every 16-lane ds_read_b128 group conflict-free for the MFMA fragment
// pattern (16 rows x one chunk).  Block ids are remapped XCD-aware and
// grouped along M so the 8 private L2s each see a compact panel of A and B.
//
// Generic path: any shape / alignment, 64x64x32 tile, guarded register
// staging with zero fill.  Same MFMA and fragment maps, slower.
#include "bk_common.hpp"

namespace bk {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef const __attribute__((address_space(1))) void* global_void_ptr;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kGemmThreads = 256;
constexpr int kRowBytes = BK * 2;                       // 128 B per tile row
constexpr int kTileElems = (BM + BN) * BK;              // A + B per stage
constexpr int kGroupM = 8;

// bijective XCD remap: blocks b, b+8, b+16.. share an XCD under round-robin
// dispatch; give each XCD a contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
  const int xcd = b % kNumXCD, q = nblocks / kNumXCD, r = nblocks % kNumXCD;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + b / kNumXCD;
}

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Stage one BMxBK (or BNxBK) tile: 16 wave-instructions per operand, 4 per
// wave.  Lane l of instruction i writes LDS bytes [l*16, l*16+16) of rows
// 8i..8i+7, i.e. row 8i + (l>>3), physical chunk l&7, fetched from the
// logical chunk that maps there.
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ g, int ld, int row0, int k0,
                                           uint16_t* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ins = wave * 4 + i;          // 0..15
    const int r = ins * 8 + (lane >> 3);   // tile row
    const int pc = lane & 7;               // physical chunk in LDS
    const int c = swz_chunk(r, pc);        // logical chunk (involution)
    const uint16_t* src = g + (int64_t)(row0 + r) * ld + k0 + c * 8;
    uint16_t* dst = lds_tile + ins * 8 * BK;  // wave-uniform base
    __builtin_amdgcn_global_load_lds((global_void_ptr)src, (lds_void_ptr)dst, 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 read_frag(const uint16_t* lds_tile, int row, int chunk) {
  const int pc = swz_chunk(row, chunk);
  return *reinterpret_cast<const bf16x8*>(lds_tile + row * BK + pc * 8);
}

template <bool OUT_BF16>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_bf16_tn_fast(const uint16_t* __restrict__ A,
                                                                     const uint16_t* __restrict__ Bt,
                                                                     void* __restrict__ C, int M, int N, int K,
                                                                     int lda, int ldb, int ldc, float alpha,
                                                                     float beta) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * kTileElems];  // 64 KiB

  const int nbm = M / BM, nbn = N / BN, nblocks = nbm * nbn;
  int b = xcd_remap(blockIdx.x, nblocks);
  // grouped ordering along M for L2 reuse of the B panel
  const int group = kGroupM * nbn;
  const int first_m = (b / group) * kGroupM;
  const int gm = min(nbm - first_m, kGroupM);
  const int tm = first_m + (b % group) % gm;
  const int tn = (b % group) / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // 2x2 waves, 64x64 each

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  stage_tile(A, lda, m0, 0, smem, wave, lane);
  stage_tile(Bt, ldb, n0, 0, smem + BM * BK, wave, lane);
  __syncthreads();  // vmcnt(0) + barrier: tile 0 resident

  for (int t = 0; t < nk; ++t) {
    uint16_t* cur = smem + (t & 1) * kTileElems;
    if (t + 1 < nk) {  // prefetch next K tile into the other buffer
      uint16_t* nxt = smem + ((t + 1) & 1) * kTileElems;
      stage_tile(A, lda, m0, (t + 1) * BK, nxt, wave, lane);
      stage_tile(Bt, ldb, n0, (t + 1) * BK, nxt + BM * BK, wave, lane);
    }
    const uint16_t* tA = cur;
    const uint16_t* tB = cur + BM * BK;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const int chunk = s * 4 + (lane >> 4);
      bf16x8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag(tA, wm * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = read_frag(tB, wn * 64 + j * 16 + (lane & 15), chunk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();  // next tile landed (vmcnt(0)) and every wave done reading `cur`
  }

  // epilogue: 16x16 C/D map: col = lane & 15, row = (lane >> 4) * 4 + reg
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn * 64 + j * 16 + (lane & 15);
        float v = alpha * acc[i][j][r];
        if constexpr (OUT_BF16) {
          uint16_t* c = (uint16_t*)C + (int64_t)row * ldc + col;
          if (beta != 0.f) v += beta * bf16_bits_to_float(*c);
          *c = float_to_bf16_bits(v);
        } else {
          float* c = (float*)C + (int64_t)row * ldc + col;
          if (beta != 0.f) v += beta * *c;
          *c = v;
        }
      }
}

// ---- edge path ---------------------------------------------------------------
// The fast kernel's tiling for shapes that are not tile multiples (M, N any;
// K % 8 == 0 and 16-B aligned rows, so every 16-B chunk is all-in or
// all-out of range).  Operands are read through buffer resources whose
// extent ends at the operand's last row: rows past M / N fall outside it and
// the load returns zeros; a chunk past K gets an offset beyond the extent,
// zeros again.  Stores are masked.  Same LDS image, swizzle, MFMA schedule.
constexpr uint32_t kOob = 0x80000000u;  // past any extent this path builds

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const uint16_t* g, int ld, int row0, int rows_total) {
  const uint16_t* base = g + (int64_t)row0 * ld;
  const int64_t span = (int64_t)(rows_total - row0) * ld * 2;
  const uint64_t addr = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)addr);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32));
  const uint32_t bytes = __builtin_amdgcn_readfirstlane(span > 0x7fffffffll ? 0x7fffffffu : (uint32_t)span);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}

__device__ __forceinline__ void stage_tile_edge(__amdgpu_buffer_rsrc_t rsrc, int ld, int K, int k0, uint16_t* lds_tile,
                                                int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ins = wave * 4 + i;
    const int r = ins * 8 + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    const int k = k0 + c * 8;
    const uint32_t voff = k < K ? (uint32_t)(r * ld + k) * 2u : kOob;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_ptr)(lds_tile + ins * 8 * BK), 16, voff, 0, 0, 0);
  }
}

template <bool OUT_BF16>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_bf16_tn_edge(const uint16_t* __restrict__ A,
                                                                     const uint16_t* __restrict__ Bt,
                                                                     void* __restrict__ C, int M, int N, int K,
                                                                     int lda, int ldb, int ldc, float alpha,
                                                                     float beta) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * kTileElems];

  const int nbm = (M + BM - 1) / BM, nbn = (N + BN - 1) / BN, nblocks = nbm * nbn;
  int b = xcd_remap(blockIdx.x, nblocks);
  const int group = kGroupM * nbn;
  const int first_m = (b / group) * kGroupM;
  const int gm = min(nbm - first_m, kGroupM);
  const int tm = first_m + (b % group) % gm;
  const int tn = (b % group) / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const __amdgpu_buffer_rsrc_t ra = tile_rsrc(A, lda, m0, M), rb = tile_rsrc(Bt, ldb, n0, N);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  stage_tile_edge(ra, lda, K, 0, smem, wave, lane);
  stage_tile_edge(rb, ldb, K, 0, smem + BM * BK, wave, lane);
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    uint16_t* cur = smem + (t & 1) * kTileElems;
    if (t + 1 < nk) {
      uint16_t* nxt = smem + ((t + 1) & 1) * kTileElems;
      stage_tile_edge(ra, lda, K, (t + 1) * BK, nxt, wave, lane);
      stage_tile_edge(rb, ldb, K, (t + 1) * BK, nxt + BM * BK, wave, lane);
    }
    const uint16_t* tA = cur;
    const uint16_t* tB = cur + BM * BK;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const int chunk = s * 4 + (lane >> 4);
      bf16x8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag(tA, wm * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = read_frag(tB, wn * 64 + j * 16 + (lane & 15), chunk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn * 64 + j * 16 + (lane & 15);
        if (row >= M || col >= N) continue;
        float v = alpha * acc[i][j][r];
        if constexpr (OUT_BF16) {
          uint16_t* c = (uint16_t*)C + (int64_t)row * ldc + col;
          if (beta != 0.f) v += beta * bf16_bits_to_float(*c);
          *c = float_to_bf16_bits(v);
        } else {
          float* c = (float*)C + (int64_t)row * ldc + col;
          if (beta != 0.f) v += beta * *c;
          *c = v;
        }
      }
}

// ---- skinny strip: C[:, 0:r] for r <= 16 columns -------------------------------
// What is left right of the 256-multiples when N % 256 is tiny (4097 = 16 *
// 256 + 1): a GEMV-shaped sliver whose cost is reading A once.  One wave per
// two rows of A, 16-B chunks (64 lanes x 8 = 512 K-columns per step), the r
// rows of Bt from L2, f32 FMAs, a cross-lane sum per output.
constexpr int kSkinnyCols = 16, kSkinnyRows = 2;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <bool OUT_BF16>
__global__ __launch_bounds__(256) void gemm_bf16_tn_skinny(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                                                           void* __restrict__ C, int M, int r, int K, int lda, int ldb,
                                                           int ldc, float alpha, float beta) {
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kSkinnyRows;
  if (row0 >= M) return;  // whole wave
  float acc[kSkinnyRows][kSkinnyCols];
#pragma unroll
  for (int i = 0; i < kSkinnyRows; ++i)
#pragma unroll
    for (int j = 0; j < kSkinnyCols; ++j) acc[i][j] = 0.f;
  // four K steps' loads in flight per lane (the GEMV shape is latency-bound:
  // 4096^2 . 4096 ran 9.4 us with one step at a time); the FMAs still run
  // step by step, so the sums are the one-step loop's
  constexpr int KB = 4;
  int k = lane * 8;
  for (; k + (KB - 1) * 512 < K; k += KB * 512) {
    uint4 qa[KB][kSkinnyRows];
#pragma unroll
    for (int s = 0; s < KB; ++s)
#pragma unroll
      for (int i = 0; i < kSkinnyRows; ++i) {
        const int64_t row = min(row0 + i, (int64_t)M - 1);
        qa[s][i] = *reinterpret_cast<const uint4*>(A + row * lda + k + s * 512);
      }
#pragma unroll
    for (int j = 0; j < kSkinnyCols; ++j) {
      if (j >= r) break;
      uint4 qb[KB];
#pragma unroll
      for (int s = 0; s < KB; ++s) qb[s] = *reinterpret_cast<const uint4*>(Bt + (int64_t)j * ldb + k + s * 512);
#pragma unroll
      for (int s = 0; s < KB; ++s) {
        const uint32_t wb[4] = {qb[s].x, qb[s].y, qb[s].z, qb[s].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float b0 = bf16_bits_to_float((uint16_t)(wb[e] & 0xffff)), b1 = bf16_bits_to_float((uint16_t)(wb[e] >> 16));
#pragma unroll
          for (int i = 0; i < kSkinnyRows; ++i) {
            const uint32_t wa = e == 0 ? qa[s][i].x : e == 1 ? qa[s][i].y : e == 2 ? qa[s][i].z : qa[s][i].w;
            acc[i][j] += bf16_bits_to_float((uint16_t)(wa & 0xffff)) * b0 + bf16_bits_to_float((uint16_t)(wa >> 16)) * b1;
          }
        }
      }
    }
  }
  for (; k < K; k += 512) {  // K % 8 == 0: chunks are whole
    float a[kSkinnyRows][8];
#pragma unroll
    for (int i = 0; i < kSkinnyRows; ++i) {
      const int64_t row = min(row0 + i, (int64_t)M - 1);  // (a clamped duplicate row is never stored)
      const uint4 q = *reinterpret_cast<const uint4*>(A + row * lda + k);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[i][2 * e] = bf16_bits_to_float((uint16_t)(w[e] & 0xffff));
        a[i][2 * e + 1] = bf16_bits_to_float((uint16_t)(w[e] >> 16));
      }
    }
#pragma unroll
    for (int j = 0; j < kSkinnyCols; ++j) {
      if (j >= r) break;
      const uint4 q = *reinterpret_cast<const uint4*>(Bt + (int64_t)j * ldb + k);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float b0 = bf16_bits_to_float((uint16_t)(w[e] & 0xffff)), b1 = bf16_bits_to_float((uint16_t)(w[e] >> 16));
#pragma unroll
        for (int i = 0; i < kSkinnyRows; ++i) acc[i][j] += a[i][2 * e] * b0 + a[i][2 * e + 1] * b1;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kSkinnyRows; ++i) {
    const int64_t row = row0 + i;
#pragma unroll
    for (int j = 0; j < kSkinnyCols; ++j) {
      if (j >= r) break;
      const float s = wave_sum(acc[i][j]);
      if (lane == 0 && row < M) {
        float v = alpha * s;
        if constexpr (OUT_BF16) {
          uint16_t* c = (uint16_t*)C + row * ldc + j;
          if (beta != 0.f) v += beta * bf16_bits_to_float(*c);
          *c = float_to_bf16_bits(v);
        } else {
          float* c = (float*)C + row * ldc + j;
          if (beta != 0.f) v += beta * *c;
          *c = v;
        }
      }
    }
  }
}

// ---- generic path ------------------------------------------------------------
constexpr int GBM = 64, GBN = 64, GBK = 32;

template <bool OUT_BF16>
__global__ __launch_bounds__(256) void gemm_bf16_tn_generic(const uint16_t* __restrict__ A,
                                                            const uint16_t* __restrict__ Bt, void* __restrict__ C,
                                                            int M, int N, int K, int lda, int ldb, int ldc,
                                                            float alpha, float beta) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[GBM * (GBK + 8)];
  __shared__ __attribute__((aligned(16))) uint16_t sB[GBN * (GBK + 8)];
  constexpr int LD = GBK + 8;  // +16 B pad per row breaks the power-of-2 stride
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // 2x2 waves of 32x32
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += GBK) {
    // 64 rows x 32 cols per operand = 2048 elems; 256 threads x 8 elems
    {
      const int r = tid >> 2, c = (tid & 3) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int gk = k0 + c + e;
        const int ga = m0 + r, gb = n0 + r;
        sA[r * LD + c + e] = (ga < M && gk < K) ? A[(int64_t)ga * lda + gk] : (uint16_t)0;
        sB[r * LD + c + e] = (gb < N && gk < K) ? Bt[(int64_t)gb * ldb + gk] : (uint16_t)0;
      }
    }
    __syncthreads();
    bf16x8 af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wm * 32 + i * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        uint16_t bits = sA[row * LD + (lane >> 4) * 8 + e];
        af[i][e] = __builtin_bit_cast(__bf16, bits);
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        uint16_t bits = sB[row * LD + (lane >> 4) * 8 + e];
        bfr[j][e] = __builtin_bit_cast(__bf16, bits);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn * 32 + j * 16 + (lane & 15);
        if (row < M && col < N) {
          float v = alpha * acc[i][j][r];
          if constexpr (OUT_BF16) {
            uint16_t* c = (uint16_t*)C + (int64_t)row * ldc + col;
            if (beta != 0.f) v += beta * bf16_bits_to_float(*c);
            *c = float_to_bf16_bits(v);
          } else {
            float* c = (float*)C + (int64_t)row * ldc + col;
            if (beta != 0.f) v += beta * *c;
            *c = v;
          }
        }
      }
}

// Tiled transpose of a bf16 matrix (rows x cols, row-major, ld) into
// out[cols x rows]; used to turn a row-major B[K,N] into Bt[N,K].
__global__ __launch_bounds__(256) void transpose_bf16(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                      int rows, int cols, int ld_in, int ld_out) {
  __shared__ uint16_t tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  for (int y = ty; y < 64; y += 4) {
    const int r = r0 + y, c = c0 + tx;
    if (r < rows && c < cols) tile[y][tx] = in[(int64_t)r * ld_in + c];
  }
  __syncthreads();
  for (int y = ty; y < 64; y += 4) {
    const int c = c0 + y, r = r0 + tx;  // out row = input column
    if (c < cols && r < rows) out[(int64_t)c * ld_out + r] = tile[tx][y];
  }
}

// Vectorised transpose for 8-aligned shapes: each lane moves an 8x8 block
// with eight 16-B loads and eight 16-B stores and swaps the halfwords in
// registers (v_perm), so there is no LDS round trip and no barrier.  Per load
// instruction a wave touches 8 input rows x 128 B (8 lanes per row), per store
// 8 output rows x 128 B: whole cache lines both ways, where the tiled kernel
// above moves 2 B per lane (128 B per wave instruction).  Block = 4 waves side
// by side along the columns: a 64 x 256 input tile.
__global__ __launch_bounds__(256) void transpose_bf16_v8(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                         int rows, int cols, int ld_in, int ld_out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.y * 64 + (lane >> 3) * 8;
  const int c = blockIdx.x * 256 + wave * 64 + (lane & 7) * 8;
  if (r >= rows || c >= cols) return;  // rows, cols are multiples of 8: a block is all in or all out
  uint4 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const uint4*>(in + (int64_t)(r + i) * ld_in + c);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // output row c + j = input column j: halfword j of each of the 8 rows
    uint32_t w[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const uint32_t* a = reinterpret_cast<const uint32_t*>(&v[2 * m]);
      const uint32_t* b = reinterpret_cast<const uint32_t*>(&v[2 * m + 1]);
      // bytes of {b:a}: even j takes the low halfwords, odd j the high ones
      w[m] = __builtin_amdgcn_perm(b[j >> 1], a[j >> 1], (j & 1) ? 0x07060302u : 0x05040100u);
    }
    *reinterpret_cast<uint4*>(out + (int64_t)(c + j) * ld_out + r) = uint4{w[0], w[1], w[2], w[3]};
  }
}

// The same 8x8 register-block transpose fused with the f32/f64 -> bf16
// conversion the TN GEMM needs for a non-bf16 row-major B: one pass reads
// the wide input and writes Bt in bf16 (cast-then-transpose read it, wrote a
// bf16 copy, read that and wrote Bt).  Rounding is the cast kernel's
// ((float) then RNE to bf16), so the result is bitwise that of the two passes.
template <typename T>
__global__ __launch_bounds__(256) void transpose_to_bf16_v8(const T* __restrict__ in, uint16_t* __restrict__ out,
                                                            int rows, int cols, int ld_in, int ld_out) {
  constexpr int kVec = 16 / sizeof(T);  // elements per 16-B load
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.y * 64 + (lane >> 3) * 8;
  const int c = blockIdx.x * 256 + wave * 64 + (lane & 7) * 8;
  if (r >= rows || c >= cols) return;
  uint16_t h[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    T x[8];
#pragma unroll
    for (int q = 0; q < 8 / kVec; ++q)
      *reinterpret_cast<uint4*>(&x[q * kVec]) = *reinterpret_cast<const uint4*>(in + (int64_t)(r + i) * ld_in + c + q * kVec);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (sizeof(T) == 8)
        h[i][j] = double_to_bf16_bits(x[j]);
      else
        h[i][j] = float_to_bf16_bits(x[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t w[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) w[m] = (uint32_t)h[2 * m][j] | ((uint32_t)h[2 * m + 1][j] << 16);
    *reinterpret_cast<uint4*>(out + (int64_t)(c + j) * ld_out + r) = uint4{w[0], w[1], w[2], w[3]};
  }
}

// Same-dtype transpose of 4- and 8-byte elements (f32/i32, f64/i64): the
// 8x8 register-block scheme with 2 (4 B) or 4 (8 B) 16-B loads and stores per
// block row, so DeviceArray.T of a wide array no longer goes through the host.
template <typename T>
__global__ __launch_bounds__(256) void transpose_wide_v8(const T* __restrict__ in, T* __restrict__ out, int rows,
                                                         int cols, int ld_in, int ld_out) {
  constexpr int kVec = 16 / sizeof(T);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.y * 64 + (lane >> 3) * 8;
  const int c = blockIdx.x * 256 + wave * 64 + (lane & 7) * 8;
  if (r >= rows || c >= cols) return;
  T v[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8 / kVec; ++q)
      *reinterpret_cast<uint4*>(&v[i][q * kVec]) = *reinterpret_cast<const uint4*>(in + (int64_t)(r + i) * ld_in + c + q * kVec);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    T w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = v[i][j];
#pragma unroll
    for (int q = 0; q < 8 / kVec; ++q)
      *reinterpret_cast<uint4*>(out + (int64_t)(c + j) * ld_out + r + q * kVec) = *reinterpret_cast<const uint4*>(&w[q * kVec]);
  }
}

// any shape / alignment: one element per thread, writes coalesced
template <typename T>
__global__ __launch_bounds__(256) void transpose_wide_scalar(const T* __restrict__ in, T* __restrict__ out, int rows,
                                                             int cols, int ld_in, int ld_out) {
  const int64_t n = (int64_t)rows * cols, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int oc = (int)(i / rows), orow = (int)(i % rows);  // out[oc][orow] = in[orow][oc]
    out[(int64_t)oc * ld_out + orow] = in[(int64_t)orow * ld_in + oc];
  }
}

bool gemm256_ok(int M, int N, int K, int lda, int ldb, int ldc, bool out_bf16);  // gemm_bf16_256.hip
void launch_gemm256(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
                    float beta, bool out_bf16, hipStream_t stream, int which);
bool gemm256_edge_ok(int M, int N, int K, int lda, int ldb);
bool gemm256_nn_ok(int M, int N, int K, int lda, int ldb, int ldc, bool out_bf16);
void launch_gemm256_nn(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                       float alpha, float beta, bool out_bf16, hipStream_t stream);
void launch_gemm256_edge(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                         float alpha, float beta, bool out_bf16, hipStream_t stream);

}  // namespace bk

using namespace bk;

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

BK_API int bk_gemm_bf16_fast_ok(int M, int N, int K, int lda, int ldb) {
  return M > 0 && N > 0 && K > 0 && M % BM == 0 && N % BN == 0 && K % BK == 0 && lda % 8 == 0 && ldb % 8 == 0;
}

// the edge kernel: any M, N; 16-B chunks (K, ld multiples of 8); a 128-row
// tile's byte extent within the 31-bit buffer offsets
// the skinny kernel's 16-B loads: K, lda, ldb multiples of 8 elements
static bool skinny_ok(const void* A, const void* Bt, int N, int K, int lda, int ldb) {
  return aligned16(A) && aligned16(Bt) && N <= kSkinnyCols && K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0;
}

static bool edge_ok(int M, int N, int K, int lda, int ldb) {
  return M > 0 && N > 0 && K > 0 && K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         (int64_t)BM * lda * 2 < 0x7fffffffll && (int64_t)BN * ldb * 2 < 0x7fffffffll;
}

// Kernel choice: the 256x256 phase-pipelined kernel when the shape fills at
// least half the chip with 256^2 tiles, the 128x128 kernel for smaller
// aligned shapes (4x the blocks), the guarded generic kernel otherwise.
// Shapes that are not tile multiples take the edge kernel (128x128 tiles,
// zero-filling buffer loads, masked stores) when K and the leading
// dimensions are multiples of 8; only the rest reach the generic kernel.
// Large non-tile-multiple shapes take the 4-wave 256x256 kernel in its edge
// mode (variant 7; K % 8 == 0) when they fill the chip.
// variant: 0 = auto, 1 = generic, 2 = 128x128, 3 = 256x256 (4-wave or 8-wave
// by K), 4 = 256x256 8-wave, 5 = 256x256 4-wave, 6 = 128x128 edge, 7 = 256x256
// 4-wave edge, 8 = skinny (N <= 16: a matrix-vector product) (benchmarks, tests).
static int auto_variant(bool ok256, bool ok128, bool okedge, bool ok256e, bool okskinny, int M, int N) {
  if (okskinny) return 8;  // GEMV-shaped (N <= 16): read A once, no mostly-empty tiles
  const int64_t tiles256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  if (ok256 && (M / 256) * (N / 256) >= 128) return 3;
  if (ok128) return 2;
  if (ok256e && tiles256 >= 128) return 7;
  return okedge ? 6 : 1;
}

BK_API int bk_gemm_bf16_tn_variant(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb,
                                   int ldc, float alpha, float beta, int out_dtype, int variant, hipStream_t stream) {
  if (!A || !Bt || !C || M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < K || ldc < N) return kBadArgument;
  if (out_dtype != kBF16 && out_dtype != kF32) return kBadArgument;
  const bool al = aligned16(A) && aligned16(Bt);
  const bool ok128 = al && bk_gemm_bf16_fast_ok(M, N, K, lda, ldb);
  const bool ok256 = al && aligned16(C) && gemm256_ok(M, N, K, lda, ldb, ldc, out_dtype == kBF16);
  const bool okedge = al && edge_ok(M, N, K, lda, ldb);
  const bool ok256e = al && gemm256_edge_ok(M, N, K, lda, ldb);
  const bool okskinny = skinny_ok(A, Bt, N, K, lda, ldb);
  if (variant == 0) variant = auto_variant(ok256, ok128, okedge, ok256e, okskinny, M, N);
  if ((variant >= 3 && variant <= 5 && !ok256) || (variant == 2 && !ok128) || (variant == 6 && !okedge) ||
      (variant == 7 && !ok256e) || (variant == 8 && !okskinny) || variant < 1 || variant > 8)
    return kBadArgument;
  const bool bf = out_dtype == kBF16;
  if (variant == 8) {
    const unsigned g = (unsigned)((M + 4 * kSkinnyRows - 1) / (4 * kSkinnyRows));
    if (bf)
      gemm_bf16_tn_skinny<true><<<g, 256, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K, lda, ldb,
                                                       ldc, alpha, beta);
    else
      gemm_bf16_tn_skinny<false><<<g, 256, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K, lda, ldb,
                                                        ldc, alpha, beta);
  } else if (variant == 7) {
    // a remainder of <= 64 rows / columns past the 256-multiples would cost a
    // whole extra wave of mostly-empty 256^2 tiles (4095 x 4097: 272 tiles on
    // 256 CUs); it goes to the 128^2 edge kernel as a strip after the main
    // block instead
    const int es = bf ? 2 : 4;
    const int rm = M % 256, rn = N % 256;
    const int Mm = (rm && rm <= 64 && M > 256) ? M - rm : M;
    const int Nm = (rn && rn <= 64 && N > 256) ? N - rn : N;
    launch_gemm256_edge(A, Bt, C, Mm, Nm, K, lda, ldb, ldc, alpha, beta, bf, stream);
    auto strip = [&](const void* a, const void* b, void* c, int m, int n) {
      if (n <= kSkinnyCols) {  // a sliver of columns: read A once, GEMV-style
        const unsigned g = (unsigned)((m + 4 * kSkinnyRows - 1) / (4 * kSkinnyRows));
        if (bf)
          gemm_bf16_tn_skinny<true><<<g, 256, 0, stream>>>((const uint16_t*)a, (const uint16_t*)b, c, m, n, K, lda, ldb,
                                                           ldc, alpha, beta);
        else
          gemm_bf16_tn_skinny<false><<<g, 256, 0, stream>>>((const uint16_t*)a, (const uint16_t*)b, c, m, n, K, lda,
                                                            ldb, ldc, alpha, beta);
        return;
      }
      const unsigned grid = (unsigned)(((m + BM - 1) / BM) * ((n + BN - 1) / BN));
      if (bf)
        gemm_bf16_tn_edge<true><<<grid, kGemmThreads, 0, stream>>>((const uint16_t*)a, (const uint16_t*)b, c, m, n, K,
                                                                   lda, ldb, ldc, alpha, beta);
      else
        gemm_bf16_tn_edge<false><<<grid, kGemmThreads, 0, stream>>>((const uint16_t*)a, (const uint16_t*)b, c, m, n, K,
                                                                    lda, ldb, ldc, alpha, beta);
    };
    if (Nm < N)  // right strip, full height (the corner included)
      strip(A, (const uint16_t*)Bt + (int64_t)Nm * ldb, (char*)C + (int64_t)Nm * es, M, N - Nm);
    if (Mm < M)  // bottom strip left of it
      strip((const uint16_t*)A + (int64_t)Mm * lda, Bt, (char*)C + (int64_t)Mm * ldc * es, M - Mm, Nm);
  } else if (variant == 6) {
    const unsigned grid = (unsigned)(((M + BM - 1) / BM) * ((N + BN - 1) / BN));
    if (bf)
      gemm_bf16_tn_edge<true><<<grid, kGemmThreads, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K,
                                                                 lda, ldb, ldc, alpha, beta);
    else
      gemm_bf16_tn_edge<false><<<grid, kGemmThreads, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N,
                                                                  K, lda, ldb, ldc, alpha, beta);
  } else if (variant >= 3) {
    launch_gemm256(A, Bt, C, M, N, K, lda, ldb, ldc, alpha, beta, bf, stream, variant - 3);
  } else if (variant == 2) {
    const unsigned grid = (unsigned)((M / BM) * (N / BN));
    if (bf)
      gemm_bf16_tn_fast<true><<<grid, kGemmThreads, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K,
                                                                 lda, ldb, ldc, alpha, beta);
    else
      gemm_bf16_tn_fast<false><<<grid, kGemmThreads, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N,
                                                                  K, lda, ldb, ldc, alpha, beta);
  } else {
    dim3 grid((N + GBN - 1) / GBN, (M + GBM - 1) / GBM);
    if (bf)
      gemm_bf16_tn_generic<true><<<grid, 256, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K, lda,
                                                           ldb, ldc, alpha, beta);
    else
      gemm_bf16_tn_generic<false><<<grid, 256, 0, stream>>>((const uint16_t*)A, (const uint16_t*)Bt, C, M, N, K, lda,
                                                            ldb, ldc, alpha, beta);
  }
  return launch_status();
}

// Which kernel `variant 0` resolves to for these operands (diagnostics).
BK_API int bk_gemm_bf16_pick(const void* A, const void* Bt, const void* C, int M, int N, int K, int lda, int ldb,
                             int ldc, int out_dtype) {
  const bool al = aligned16(A) && aligned16(Bt);
  const bool ok128 = al && bk_gemm_bf16_fast_ok(M, N, K, lda, ldb);
  const bool ok256 = al && aligned16(C) && gemm256_ok(M, N, K, lda, ldb, ldc, out_dtype == kBF16);
  return auto_variant(ok256, ok128, al && edge_ok(M, N, K, lda, ldb), al && gemm256_edge_ok(M, N, K, lda, ldb),
                      skinny_ok(A, Bt, N, K, lda, ldb), M, N);
}

// C = alpha * A . B + beta * C with B stored [K][N] (leading dimension ldb):
// the 4-wave 256x256 kernel reading B through transposed LDS reads, no
// transpose pass.  Tile-multiple shapes (M, N % 256, K % 64) with 16-B
// aligned operands only: kBadArgument otherwise (callers transpose B and use
// bk_gemm_bf16_tn).
BK_API int bk_gemm_bf16_nn_ok(const void* A, const void* B, const void* C, int M, int N, int K, int lda, int ldb,
                              int ldc, int out_dtype) {
  return A && B && C && (out_dtype == kBF16 || out_dtype == kF32) && lda >= K && ldc >= N && aligned16(A) &&
         aligned16(B) && aligned16(C) && gemm256_nn_ok(M, N, K, lda, ldb, ldc, out_dtype == kBF16);
}

BK_API int bk_gemm_bf16_nn(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                           float alpha, float beta, int out_dtype, hipStream_t stream) {
  if (!bk_gemm_bf16_nn_ok(A, B, C, M, N, K, lda, ldb, ldc, out_dtype)) return kBadArgument;
  launch_gemm256_nn(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, out_dtype == kBF16, stream);
  return launch_status();
}

// C = alpha * A . Bt^T + beta * C.  out_dtype: kBF16 or kF32.
BK_API int bk_gemm_bf16_tn(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                           float alpha, float beta, int out_dtype, hipStream_t stream) {
  return bk_gemm_bf16_tn_variant(A, Bt, C, M, N, K, lda, ldb, ldc, alpha, beta, out_dtype, 0, stream);
}

BK_API int bk_transpose_bf16(const void* in, void* out, int rows, int cols, int ld_in, int ld_out,
                             hipStream_t stream) {
  if (!in || !out || rows <= 0 || cols <= 0 || ld_in < cols || ld_out < rows) return kBadArgument;
  if (rows % 8 == 0 && cols % 8 == 0 && ld_in % 8 == 0 && ld_out % 8 == 0 && aligned16(in) && aligned16(out)) {
    dim3 grid((cols + 255) / 256, (rows + 63) / 64);
    transpose_bf16_v8<<<grid, 256, 0, stream>>>((const uint16_t*)in, (uint16_t*)out, rows, cols, ld_in, ld_out);
  } else {
    dim3 grid((cols + 63) / 64, (rows + 63) / 64);
    transpose_bf16<<<grid, 256, 0, stream>>>((const uint16_t*)in, (uint16_t*)out, rows, cols, ld_in, ld_out);
  }
  return launch_status();
}

// out[cols x rows] (bf16) = transpose of in[rows x cols] (src_dtype kBF16,
// kF32 or kF64).  Wide inputs need the 8-aligned, 16-B aligned shape of the
// vector kernel (kBadArgument otherwise: the caller casts, then transposes).
BK_API int bk_transpose_to_bf16(int src_dtype, const void* in, void* out, int rows, int cols, int ld_in, int ld_out,
                                hipStream_t stream) {
  if (src_dtype == kBF16) return bk_transpose_bf16(in, out, rows, cols, ld_in, ld_out, stream);
  if (!in || !out || rows <= 0 || cols <= 0 || ld_in < cols || ld_out < rows) return kBadArgument;
  if (src_dtype != kF32 && src_dtype != kF64) return kBadArgument;
  if (rows % 8 || cols % 8 || ld_in % 8 || ld_out % 8 || !aligned16(in) || !aligned16(out)) return kBadArgument;
  dim3 grid((cols + 255) / 256, (rows + 63) / 64);
  if (src_dtype == kF32)
    transpose_to_bf16_v8<float><<<grid, 256, 0, stream>>>((const float*)in, (uint16_t*)out, rows, cols, ld_in, ld_out);
  else
    transpose_to_bf16_v8<double><<<grid, 256, 0, stream>>>((const double*)in, (uint16_t*)out, rows, cols, ld_in, ld_out);
  return launch_status();
}

// out[cols x rows] = transpose of in[rows x cols].  dst_dtype kBF16 converts
// (bk_transpose_to_bf16); dst_dtype == src_dtype moves the bits (2-, 4- or
// 8-byte elements).
BK_API int bk_transpose(int src_dtype, int dst_dtype, const void* in, void* out, int rows, int cols, int ld_in,
                        int ld_out, hipStream_t stream) {
  if (dst_dtype == kBF16) return bk_transpose_to_bf16(src_dtype, in, out, rows, cols, ld_in, ld_out, stream);
  if (dst_dtype != src_dtype) return kBadArgument;
  const int es = dtype_size(src_dtype);
  if (es == 2) return bk_transpose_bf16(in, out, rows, cols, ld_in, ld_out, stream);
  if (es != 4 && es != 8) return kBadArgument;
  if (!in || !out || rows <= 0 || cols <= 0 || ld_in < cols || ld_out < rows) return kBadArgument;
  if (rows % 8 == 0 && cols % 8 == 0 && ld_in % 8 == 0 && ld_out % 8 == 0 && aligned16(in) && aligned16(out)) {
    dim3 grid((cols + 255) / 256, (rows + 63) / 64);
    if (es == 4)
      transpose_wide_v8<uint32_t><<<grid, 256, 0, stream>>>((const uint32_t*)in, (uint32_t*)out, rows, cols, ld_in, ld_out);
    else
      transpose_wide_v8<uint64_t><<<grid, 256, 0, stream>>>((const uint64_t*)in, (uint64_t*)out, rows, cols, ld_in, ld_out);
  } else {
    const unsigned g = stream_grid((int64_t)rows * cols, 256);
    if (es == 4)
      transpose_wide_scalar<uint32_t><<<g, 256, 0, stream>>>((const uint32_t*)in, (uint32_t*)out, rows, cols, ld_in, ld_out);
    else
      transpose_wide_scalar<uint64_t><<<g, 256, 0, stream>>>((const uint64_t*)in, (uint64_t*)out, rows, cols, ld_in, ld_out);
  }
  return launch_status();
}
