// The 4-wave 256x256 kernel's edge (any M x N, ragged K) and [K][N]-B
// instantiations, in their own translation unit: compiled next to the
// shipped aligned kernel they changed its register allocation (one VGPR
// spilled in the main loop), alone it is the same code as before.
#include "gemm256w4_impl.hpp"

namespace bk {

constexpr long long kShippedW4x = g4::kAsmMfma | g4::kInterleave;
// the edge kernel runs the aligned kernel's two-barrier schedule and
// non-temporal stores (gemm_bf16_256.hip kShippedW4; tools/gemm_lab.py
// w4_asm_twobar_ntstore_edge).  (The [K][N] kernel keeps its schedule: with
// kNtStore its f32-output instance spills 4 VGPRs.)
constexpr long long kShippedW4Edge = kShippedW4x | g4::kTwoBar | g4::kTwoBarG10 | g4::kNtStore;

// the 4-wave 256x256 kernel on any M x N (K a multiple of 64): ragged
// borders read zeros and store under a mask (g4::kEdge)
bool gemm256_edge_ok(int M, int N, int K, int lda, int ldb) { return g4::edge_ok(M, N, K, lda, ldb); }

void launch_gemm256_edge(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                         float alpha, float beta, bool out_bf16, hipStream_t stream) {
  g4::launch<kShippedW4Edge | g4::kEdge>(A, Bt, C, M, N, K, lda, ldb, ldc, alpha, beta, out_bf16, stream);
}

// C = A . B with B stored [K][N] (no transpose pass): the 4-wave kernel with
// transposed LDS reads of B (g4::kNN)
bool gemm256_nn_ok(int M, int N, int K, int lda, int ldb, int ldc, bool out_bf16) {
  return g4::nn_ok(M, N, K, lda, ldb, ldc, out_bf16);
}

void launch_gemm256_nn(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                       float alpha, float beta, bool out_bf16, hipStream_t stream) {
  g4::launch<kShippedW4x | g4::kNN>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, out_bf16, stream);
}

}  // namespace bk
