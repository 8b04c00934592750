// GEMM schedule lab: every 256x256 schedule variant in ONE binary, so
// tools/gemm_lab.py can A/B them interleaved in one process (guide §5.4
// rules 19/24).  Not part of libbeekern.
#include "../../csrc/kernels/gemm256_impl.hpp"
#include "../../csrc/kernels/gemm256w4_impl.hpp"

using namespace bk;

namespace {
constexpr int kLabOpts[] = {
    g256::kOptRound1,           // 0: round-1 schedule (shipped until a variant wins)
    g256::kOptKeepB0,           // 1: B0 kept in registers, every half >= 5 phases ahead
    0,                          // 2: round-1 without the wave-group stagger
    g256::kKeepB0,              // 3: keep-B0 without the stagger
    g256::kStagger | g256::kSameTile,  // 4: DIAGNOSTIC round-1 on L2-resident operands (wrong C)
    g256::kOptKeepB0 | g256::kSameTile,  // 5: DIAGNOSTIC keep-B0 on L2-resident operands (wrong C)
};
template <int I>
void run(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, bool bf,
         hipStream_t s) {
  g256::launch<kLabOpts[I]>(A, B, C, M, N, K, lda, ldb, ldc, 1.0f, 0.0f, bf, s);
}
}  // namespace

// 4-wave 128x128-per-wave kernel options, lab ids 6..
constexpr long long kW4Opts[] = {0, g4::kPinOrder, g4::kInterleave, g4::kNoCarry, g4::kDirectStore,
                           g4::kAsmMfma | g4::kInterleave, g4::kAsmMfma | g4::kNoCarry,
                           g4::kAsmMfma | g4::kInterleave | g4::kEarlyGlds,
                           g4::kAsmMfma | g4::kInterleave | g4::kReadsEarly,
                           g4::kAsmMfma | g4::kInterleave | g4::kReadsEarly | g4::kEarlyGlds,
                           g4::kAsmMfma | g4::kInterleave | g4::kGroup2,
                           g4::kAsmMfma | g4::kInterleave | g4::kGroup8,
                           g4::kAsmMfma | g4::kInterleave | g4::kGroup16,
                           g4::kAsmMfma | g4::kInterleave | g4::kThreeBar,
                           g4::kAsmMfma | g4::kInterleave | g4::kThreeBar | g4::kGroup8,
                           g4::kAsmMfma | g4::kInterleave | g4::kThreeBar | g4::kEdge,
                           g4::kAsmMfma | g4::kInterleave | g4::kThreeBar | g4::kSpread,
                           g4::kAsmMfma | g4::kInterleave | g4::kThreeBar | g4::kSpread | g4::kEdge,
                           g4::kAsmMfma | g4::kInterleave | g4::kDirectStore,
                           g4::kAsmMfma | g4::kInterleave | g4::kDiagNoEpilogue,
                           g4::kAsmMfma | g4::kInterleave | g4::kSwapAB,
                           g4::kAsmMfma | g4::kInterleave | g4::kSwapAB | g4::kEdge,
                           g4::kAsmMfma | g4::kInterleave | g4::kSwapAB | g4::kDiagNoEpilogue,
                           g4::kAsmMfma | g4::kInterleave | g4::kAltSimd,
                           g4::kAsmMfma | g4::kInterleave | g4::kAltSimd | g4::kSwapAB,
                           g4::kAsmMfma | g4::kInterleave | g4::kAltSimd | g4::kEarlyGlds,
                           g4::kAsmMfma | g4::kInterleave | g4::kDiagStamps,
                           g4::kAsmMfma | g4::kInterleave | g4::kDiagStamps | g4::kDiagNoGlds,
                           g4::kAsmMfma | g4::kInterleave | g4::kDiagStamps | g4::kSplitGlds,
                           g4::kAsmMfma | g4::kInterleave | g4::kSplitGlds,
                           g4::kAsmMfma | g4::kInterleave | g4::kDiagNoGlds,
                           g4::kAsmMfma | g4::kInterleave | g4::kSpacedMem,
                           g4::kAsmMfma | g4::kInterleave | g4::kDiagStamps | g4::kSpacedMem,
                           g4::kAsmMfma | g4::kInterleave | g4::kSpacedMem | g4::kEdge,
                           g4::kAsmMfma | g4::kInterleave | g4::kDiagStamps | g4::kDiagMfmaOnly,
                           g4::kAsmMfma | g4::kInterleave | g4::kSpacedMem | g4::kConstSoff,
                           g4::kAsmMfma | g4::kInterleave | g4::kDiagStamps | g4::kSpacedMem | g4::kConstSoff,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kEdge,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG12,
                           g4::kAsmMfma | g4::kInterleave | g4::kSpacedMem | g4::kNtStore,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kNtStore,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kNtStore | g4::kEdge,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore | g4::kDiagNoVmWait,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore | g4::kDiagNoBar2,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore | g4::kDiagNoBar1,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore |
                               g4::kDiagNoVmWait | g4::kDiagNoBar2 | g4::kDiagNoBar1,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore | g4::kDiagNoReads0,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore | g4::kDiagNoGlds,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kSwapAB,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore | g4::kReads12,
                           // the shipped schedule with the other L2 tile groupings (kGroupM = 4 ships)
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore | g4::kGroup2,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore | g4::kGroup8,
                           g4::kAsmMfma | g4::kInterleave | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore | g4::kGroup16};
template <int I>
void run_w4(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, bool bf,
            hipStream_t s) {
  g4::launch<kW4Opts[I]>(A, B, C, M, N, K, lda, ldb, ldc, 1.0f, 0.0f, bf, s);
}

BK_API int gemmlab_count() { return (int)(sizeof(kLabOpts) / sizeof(kLabOpts[0]) + sizeof(kW4Opts) / sizeof(kW4Opts[0])); }

BK_API int gemmlab_run(int variant, const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb,
                       int ldc, int out_bf16, hipStream_t s) {
  if (!g256::ok(M, N, K, lda, ldb, ldc, out_bf16 != 0)) return kBadArgument;
  const bool bf = out_bf16 != 0;
  switch (variant) {
    case 0: run<0>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 1: run<1>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 2: run<2>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 3: run<3>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 4: run<4>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 5: run<5>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 6: run_w4<0>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 7: run_w4<1>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 8: run_w4<2>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 9: run_w4<3>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 10: run_w4<4>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 11: run_w4<5>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 12: run_w4<6>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 13: run_w4<7>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 14: run_w4<8>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 15: run_w4<9>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 16: run_w4<10>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 17: run_w4<11>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 18: run_w4<12>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 19: run_w4<13>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 20: run_w4<14>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 21: run_w4<15>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 22: run_w4<16>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 23: run_w4<17>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 24: run_w4<18>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 25: run_w4<19>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 26: run_w4<20>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 27: run_w4<21>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 28: run_w4<22>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 29: run_w4<23>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 30: run_w4<24>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 31: run_w4<25>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 32: run_w4<26>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 33: run_w4<27>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 34: run_w4<28>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 35: run_w4<29>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 36: run_w4<30>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 37: run_w4<31>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 38: run_w4<32>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 39: run_w4<33>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 40: run_w4<34>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 41: run_w4<35>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 42: run_w4<36>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 43: run_w4<37>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 44: run_w4<38>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 45: run_w4<39>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 46: run_w4<40>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 47: run_w4<41>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 48: run_w4<42>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 49: run_w4<43>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 50: run_w4<44>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 51: run_w4<45>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 52: run_w4<46>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 53: run_w4<47>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 54: run_w4<48>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 55: run_w4<49>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 56: run_w4<50>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 57: run_w4<51>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 58: run_w4<52>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 59: run_w4<53>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 60: run_w4<54>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    case 61: run_w4<55>(A, Bt, C, M, N, K, lda, ldb, ldc, bf, s); break;
    default: return kBadArgument;
  }
  return launch_status();
}
