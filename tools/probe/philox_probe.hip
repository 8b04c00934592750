// Philox4x32-10 round-multiply forms on gfx950: v_mul_hi_u32 + v_mul_lo_u32
// (two quarter-rate ops) vs one v_mad_u64_u32, in a compute-bound
// generate->reduce loop shaped like bk::rand_reduce_f64 (1e8 f64 draws).
//   hipcc --offload-arch=gfx950 -O3 tools/probe/philox_probe.hip -o /tmp/philox_probe && /tmp/philox_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <bool MAD64>
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    if constexpr (MAD64) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
      hi0 = (uint32_t)(p0 >> 32); lo0 = (uint32_t)p0; hi1 = (uint32_t)(p1 >> 32); lo1 = (uint32_t)p1;
    } else {
      hi0 = __umulhi(0xD2511F53u, c.x); lo0 = 0xD2511F53u * c.x;
      hi1 = __umulhi(0xCD9E8D57u, c.z); lo1 = 0xCD9E8D57u * c.z;
    }
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

template <bool MAD64>
__global__ __launch_bounds__(256) void gen_sq_sum(int64_t pairs, uint32_t k0, uint32_t k1, double* out) {
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < pairs; p += stride) {
    const uint4 r = philox<MAD64>(make_uint4((uint32_t)p, (uint32_t)(p >> 32), 0x62656b65u, 0u), k0, k1);
    const double a = u53(r.x, r.y), b = u53(r.z, r.w);
    acc += a * a + b * b;
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

int main() {
  const int64_t pairs = 50000000;
  double* d;
  hipMalloc(&d, sizeof(double));
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int grid : {2048, 4096, 8192, 16384}) {
    for (int v = 0; v < 2; ++v) {
      float best = 1e9f;
      double h = 0;
      for (int rep = 0; rep < 10; ++rep) {
        hipMemset(d, 0, sizeof(double));
        hipEventRecord(s);
        if (v) gen_sq_sum<true><<<grid, 256>>>(pairs, 1234u, 5678u, d);
        else gen_sq_sum<false><<<grid, 256>>>(pairs, 1234u, 5678u, d);
        hipEventRecord(e);
        hipEventSynchronize(e);
        float ms;
        hipEventElapsedTime(&ms, s, e);
        if (ms < best) best = ms;
        hipMemcpy(&h, d, sizeof(double), hipMemcpyDeviceToHost);
      }
      printf("{\"grid\": %d, \"form\": \"%s\", \"best_us\": %.2f, \"mean_sq\": %.6f}\n", grid, v ? "mad_u64_u32" : "mul_hi+mul_lo",
             best * 1e3, h / (2.0 * pairs));
    }
  }
  return 0;
}
