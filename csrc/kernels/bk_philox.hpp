// Philox4x32-10 and the uniform constructions shared by the RNG kernels
// (random.hip) and the fused RNG->reduce kernels (reduce.hip): one definition,
// so a fused reduction sees bit-identical values to a materialised draw.
#pragma once
#include "bk_common.hpp"

namespace bk {

struct Philox {
  static constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  static constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;

  // Each round's 32x32->64 products as ONE v_mad_u64_u32 apiece instead of
  // v_mul_hi_u32 + v_mul_lo_u32 (two quarter-rate ops): the generator is
  // VALU-bound, and tools/probe/philox_probe.hip measured a 1e8-f64
  // generate->square->sum loop 147 -> 120 us on MI355X.  Same bits.
  __device__ __forceinline__ static uint4 run(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
      const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
      const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
      // three-input XORs as ONE v_bitop3_b32 each (gfx950; truth table 0x96 =
      // a ^ b ^ c): the compiler emitted two v_xor_b32 apiece, 74 of the 183
      // instructions of rand_reduce_f64's two-Philox loop body
      c = make_uint4(__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
                     __builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0);
      k0 += W0;
      k1 += W1;
    }
    return c;
  }
};

// the 53-bit integer numpy's random() builds from two words (exact in f64)
__device__ __forceinline__ double u53_int(uint32_t a, uint32_t b) {
  return (double)(a >> 5) * 67108864.0 + (double)(b >> 6);
}
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ float u24(uint32_t a) { return (float)(a >> 8) * (1.0f / 16777216.0f); }

// stream tags: distinct counter words per distribution
constexpr uint32_t kTagUniformF64 = 0x62656b65u, kTagUniformF32 = 0x62656b66u;

}  // namespace bk
