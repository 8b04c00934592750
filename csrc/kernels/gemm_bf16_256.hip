// Shipped instantiation of the 256x256 phase-pipelined bf16 GEMM
// (gemm256_impl.hpp holds the kernel and the schedule notes).  The schedule
// chosen here is the winner of tools/gemm_lab.py on MI355X
// (profiles/r1_gemm_lab.log).
#include "gemm256_impl.hpp"

namespace bk {

constexpr int kShipped = g256::kOptRound1;

bool gemm256_ok(int M, int N, int K, int lda, int ldb, int ldc, bool out_bf16) {
  return g256::ok(M, N, K, lda, ldb, ldc, out_bf16);
}

void launch_gemm256(const void* A, const void* Bt, void* C, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
                    float beta, bool out_bf16, hipStream_t stream) {
  g256::launch<kShipped>(A, Bt, C, M, N, K, lda, ldb, ldc, alpha, beta, out_bf16, stream);
}

}  // namespace bk
