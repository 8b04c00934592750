// Counter-based Philox4x32-10 uniform generator: replaces numpy.random.rand
// in the benchmark payload (`examples/benchmark-numpy.py:20`, 1e8 f64).
//
// Element i of the stream depends only on (seed, i), never on the grid, so
// results are reproducible across launch shapes and GPU counts.  One Philox
// call yields 128 random bits = 2 f64 (numpy's 53-bit construction from two
// 32-bit draws, a>>5 and b>>6) or 4 f32 (24-bit), written with one 16-byte
// store per lane; the kernel is HBM-write bound (800 MB for 1e8 f64).
#include "bk_common.hpp"
#include "bk_philox.hpp"

namespace bk {

// out[i] = U[0,1) (f64), scaled to [lo, hi).  Each counter value -> 2 doubles.
// lo + span * u as one fma of the 53-bit integer (span * 2^-53 is exact: the
// same bits as rand_reduce_f64's fused draw, one f64 multiply fewer), and two
// counters per lane per iteration so two Philox chains overlap the stores.
template <bool NT>
__global__ __launch_bounds__(256) void philox_uniform_f64(double* __restrict__ out, int64_t n, uint32_t k0,
                                                          uint32_t k1, uint64_t offset, double lo, double span) {
  const int64_t pairs = (n + 1) / 2, full = n / 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const double s53 = span * (1.0 / 9007199254740992.0);
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; p + stride < full; p += 2 * stride) {
    const uint64_t c0 = offset + (uint64_t)p, c1 = c0 + (uint64_t)stride;
    const uint4 r0 = Philox::run(make_uint4((uint32_t)c0, (uint32_t)(c0 >> 32), kTagUniformF64, 0u), k0, k1);
    const uint4 r1 = Philox::run(make_uint4((uint32_t)c1, (uint32_t)(c1 >> 32), kTagUniformF64, 0u), k0, k1);
    st16<NT>(reinterpret_cast<double2*>(out + 2 * p),
             make_double2(fma(u53_int(r0.x, r0.y), s53, lo), fma(u53_int(r0.z, r0.w), s53, lo)));
    st16<NT>(reinterpret_cast<double2*>(out + 2 * (p + stride)),
             make_double2(fma(u53_int(r1.x, r1.y), s53, lo), fma(u53_int(r1.z, r1.w), s53, lo)));
  }
  for (; p < pairs; p += stride) {
    const uint64_t ctr = offset + (uint64_t)p;
    const uint4 r = Philox::run(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), kTagUniformF64, 0u), k0, k1);
    double2 v = make_double2(fma(u53_int(r.x, r.y), s53, lo), fma(u53_int(r.z, r.w), s53, lo));
    const int64_t i = 2 * p;
    if (i + 1 < n) {
      st16<NT>(reinterpret_cast<double2*>(out + i), v);  // 16-B store
    } else {
      out[i] = v.x;
    }
  }
}

// f32: each counter value -> 4 floats, one 16-B store.
template <bool NT>
__global__ __launch_bounds__(256) void philox_uniform_f32(float* __restrict__ out, int64_t n, uint32_t k0, uint32_t k1,
                                                          uint64_t offset, float lo, float span) {
  const int64_t quads = (n + 3) / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += stride) {
    const uint64_t ctr = offset + (uint64_t)q;
    const uint4 r = Philox::run(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), kTagUniformF32, 0u), k0, k1);
    float4 v = make_float4(lo + span * u24(r.x), lo + span * u24(r.y), lo + span * u24(r.z), lo + span * u24(r.w));
    const int64_t i = 4 * q;
    if (i + 3 < n) {
      st16<NT>(reinterpret_cast<float4*>(out + i), v);
    } else {
      const float t[4] = {v.x, v.y, v.z, v.w};
      for (int j = 0; i + j < n; ++j) out[i + j] = t[j];
    }
  }
}

// bf16: the f32 stream's values rounded once to bf16 (RNE) -- bit-identical to
// drawing f32 and casting, without the f32 buffer and the cast pass.  Each
// lane handles two counters (8 values) for one 16-B store.
__global__ __launch_bounds__(256) void philox_uniform_bf16(uint16_t* __restrict__ out, int64_t n, uint32_t k0,
                                                           uint32_t k1, uint64_t offset, float lo, float span) {
  const int64_t octs = (n + 7) / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < octs; o += stride) {
    uint16_t h[8];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const uint64_t ctr = offset + 2 * (uint64_t)o + half;
      const uint4 r = Philox::run(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), kTagUniformF32, 0u), k0, k1);
      h[4 * half + 0] = float_to_bf16_bits(lo + span * u24(r.x));
      h[4 * half + 1] = float_to_bf16_bits(lo + span * u24(r.y));
      h[4 * half + 2] = float_to_bf16_bits(lo + span * u24(r.z));
      h[4 * half + 3] = float_to_bf16_bits(lo + span * u24(r.w));
    }
    const int64_t i = 8 * o;
    if (i + 7 < n) {
      *reinterpret_cast<uint4*>(out + i) = make_uint4(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16),
                                                      h[4] | ((uint32_t)h[5] << 16), h[6] | ((uint32_t)h[7] << 16));
    } else {
      for (int j = 0; i + j < n; ++j) out[i + j] = h[j];
    }
  }
}

// Standard normal via Box-Muller on the f32 / f64 streams (for randn).
__global__ __launch_bounds__(256) void philox_normal_f32(float* __restrict__ out, int64_t n, uint32_t k0, uint32_t k1,
                                                         uint64_t offset, float mean, float std) {
  const int64_t quads = (n + 3) / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += stride) {
    const uint64_t ctr = offset + (uint64_t)q;
    const uint4 r = Philox::run(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), 0x6e6f726du, 0u), k0, k1);
    const float u1 = fmaxf(u24(r.x), 1e-12f), u2 = u24(r.y), u3 = fmaxf(u24(r.z), 1e-12f), u4 = u24(r.w);
    const float r1 = sqrtf(-2.f * __logf(u1)), r2 = sqrtf(-2.f * __logf(u3));
    float s1, c1, s2, c2;
    __sincosf(6.283185307f * u2, &s1, &c1);
    __sincosf(6.283185307f * u4, &s2, &c2);
    const float t[4] = {mean + std * r1 * c1, mean + std * r1 * s1, mean + std * r2 * c2, mean + std * r2 * s2};
    const int64_t i = 4 * q;
    if (i + 3 < n) {
      *reinterpret_cast<float4*>(out + i) = make_float4(t[0], t[1], t[2], t[3]);
    } else {
      for (int j = 0; i + j < n; ++j) out[i + j] = t[j];
    }
  }
}

__global__ __launch_bounds__(256) void philox_normal_f64(double* __restrict__ out, int64_t n, uint32_t k0, uint32_t k1,
                                                         uint64_t offset, double mean, double std) {
  const int64_t pairs = (n + 1) / 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < pairs; p += stride) {
    const uint64_t ctr = offset + (uint64_t)p;
    const uint4 r = Philox::run(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), 0x6e6f726eu, 0u), k0, k1);
    const double u1 = fmax(u53(r.x, r.y), 1e-300), u2 = u53(r.z, r.w);
    const double rad = sqrt(-2.0 * log(u1));
    double s, c;
    sincos(6.283185307179586 * u2, &s, &c);
    const int64_t i = 2 * p;
    if (i + 1 < n) {
      *reinterpret_cast<double2*>(out + i) = make_double2(mean + std * rad * c, mean + std * rad * s);
    } else {
      out[i] = mean + std * rad * c;
    }
  }
}

}  // namespace bk

using namespace bk;

// dtype: kF64, kF32 or kBF16 (the f32 stream, rounded).  `offset` advances the counter so successive draws from
// one seed never overlap (the Python side keeps the running offset).
BK_API int bk_rand_uniform(void* out, int64_t n, int dtype, uint64_t seed, uint64_t offset, double lo, double hi,
                           hipStream_t stream) {
  if (!out || n < 0) return kBadArgument;
  if (n == 0) return kOk;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  // the f64 / f32 draws take a 4x larger grid cap than the elementwise
  // kernels: 1e8 f64 (800 MB), rocprofv3 mean / min: 64 blocks/CU 146 / 139
  // us, 128: 133 / 118, 256: 133 / 121, 512: 130 / 115
  // (profiles/archive/r3_philox_grid_sweep.log)
  constexpr int kDrawBlocksPerCU = 256;
  if (dtype == kF64) {
    const int64_t pairs = (n + 1) / 2;
    const unsigned g = stream_grid(pairs, 256, kDrawBlocksPerCU);
    if (stream_nt(n * 8)) philox_uniform_f64<true><<<g, 256, 0, stream>>>((double*)out, n, k0, k1, offset, lo, hi - lo);
    else philox_uniform_f64<false><<<g, 256, 0, stream>>>((double*)out, n, k0, k1, offset, lo, hi - lo);
  } else if (dtype == kBF16) {
    const int64_t octs = (n + 7) / 8;
    philox_uniform_bf16<<<stream_grid(octs, 256), 256, 0, stream>>>((uint16_t*)out, n, k0, k1, offset, (float)lo,
                                                                     (float)(hi - lo));
  } else if (dtype == kF32) {
    const int64_t quads = (n + 3) / 4;
    const unsigned g = stream_grid(quads, 256, kDrawBlocksPerCU);
    if (stream_nt(n * 4))
      philox_uniform_f32<true><<<g, 256, 0, stream>>>((float*)out, n, k0, k1, offset, (float)lo, (float)(hi - lo));
    else
      philox_uniform_f32<false><<<g, 256, 0, stream>>>((float*)out, n, k0, k1, offset, (float)lo, (float)(hi - lo));
  } else {
    return kBadArgument;
  }
  return launch_status();
}

BK_API int bk_rand_normal(void* out, int64_t n, int dtype, uint64_t seed, uint64_t offset, double mean, double std,
                          hipStream_t stream) {
  if (!out || n < 0) return kBadArgument;
  if (n == 0) return kOk;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  if (dtype == kF64) {
    philox_normal_f64<<<stream_grid((n + 1) / 2, 256), 256, 0, stream>>>((double*)out, n, k0, k1, offset, mean, std);
  } else if (dtype == kF32) {
    philox_normal_f32<<<stream_grid((n + 3) / 4, 256), 256, 0, stream>>>((float*)out, n, k0, k1, offset, (float)mean,
                                                                         (float)std);
  } else {
    return kBadArgument;
  }
  return launch_status();
}
