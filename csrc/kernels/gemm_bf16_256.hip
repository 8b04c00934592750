// Shipped instantiations of the 256x256 bf16 GEMMs:
//   * the 8-wave phase-pipelined kernel (gemm256_impl.hpp, 128x64 per wave)
//   * the 4-wave kernel (gemm256w4_impl.hpp, 128x128 per wave) with inline-asm
//     MFMAs on AGPR accumulators and a hand-interleaved load/MFMA schedule
// Both schedules are winners of tools/gemm_lab.py on MI355X
// (profiles/archive/r1_gemm_lab.log): the 4-wave kernel issues half the LDS reads per
// MFMA and wins from K >= 256 on (4096^3: 1401 vs 1259 TFLOP/s); the 8-wave
// kernel wins short-K shapes, where the 4-wave prologue/epilogue dominate.
#include <cstring>

#include "gemm256_impl.hpp"
#include "gemm256w4_impl.hpp"

namespace bk {

constexpr int kShipped = g256::kOptRound1;
// kTwoBar | kTwoBarG10: the wait for the next K-tile's loads moved from the
// k-half boundary to group 10 of the second k-half (loads get 100-160 MFMAs
// to land instead of 68-128: SQ_WAIT_ANY 407 -> 281 cycles per wave per
// K-tile at 8192^3); kNtStore: non-temporal C stores, as hipBLASLt's NTD
// kernels.  Interleaved A/B on one MI355X (profiles/r4_gemm_pmc.md,
// tools/gemm_lab.py): 4096^3 98.9 -> 94.5 us (hipBLASLt 93.6), 8192^3
// 739 -> 705 us (hipBLASLt 671).  Before: kSpacedMem (M G M M r M groups,
// profiles/archive/r3_gemm_lab_spaced.log).
constexpr long long kShippedW4 = g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore;
constexpr int kW4MinK = 256;
// ... and again from K = 18432 on: at long K the 8-wave kernel pulls ahead
// (4096^2 x 24576: 611 vs 657 us, profiles/archive/r5_gemm_longk_probe.jsonl; the
// split f32 product's K' = 6 K: 4096^3 699 vs 780-786 us, 8192^3 5410 vs
// 5864-5895, 3072^3 427 vs 436-450, r5_gemm_f32x6_w8.jsonl); at 16384 the
// 4-wave one still leads (362 vs 419)
constexpr int kW8MinK = 18432;

bool gemm256_ok(int M, int N, int K, int lda, int ldb, int ldc, bool out_bf16) {
  return g256::ok(M, N, K, lda, ldb, ldc, out_bf16);
}

// BK_GEMM256=w8 | w4: the kernel `which == 0` resolves to for every shape
// (A/B runs of the served path: the 8-wave kernel's 214 VGPRs leave room on
// each SIMD for another sandbox's VALU-bound waves, the 4-wave kernel's 512
// do not)
static int forced_which() {
  static const int w = [] {
    const char* e = getenv("BK_GEMM256");
    return !e ? 0 : !strcmp(e, "w8") ? 1 : !strcmp(e, "w4") ? 2 : 0;
  }();
  return w;
}

// which: 0 = by shape, 1 = 8-wave, 2 = 4-wave
void launch_gemm256(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
                    float beta, bool out_bf16, hipStream_t stream, int which) {
  const bool w4_ok = g4::ok(M, N, K, lda, ldb, ldc, out_bf16);
  if (which == 0) which = forced_which();
  if (which == 0) which = (w4_ok && K >= kW4MinK && K < kW8MinK) ? 2 : 1;
  if (which == 2 && w4_ok)
    g4::launch<kShippedW4>(A, Bt, C, M, N, K, lda, ldb, ldc, alpha, beta, out_bf16, stream);
  else
    g256::launch<kShipped>(A, Bt, C, M, N, K, lda, ldb, ldc, alpha, beta, out_bf16, stream);
}

}  // namespace bk
