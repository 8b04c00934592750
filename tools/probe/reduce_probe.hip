// Streaming f64 square-sum (the materialised payload's reduction) on gfx950:
// loads in flight per lane (U) x grid size (G) x plain vs non-temporal loads,
// to find the HBM-bound configuration for bk::reduce_stage1.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/reduce_probe.hip -o tools/probe/reduce_probe && tools/probe/reduce_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

struct alignas(16) D2 { double x, y; };

template <int U, bool NT>
__global__ __launch_bounds__(256) void sqsum(const double* __restrict__ a, int64_t n, double* __restrict__ partials) {
  const int64_t nvec = n / 2;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = 0.0;
  const D2* v = reinterpret_cast<const D2*>(a);
  int64_t i = tid;
  for (; i + (U - 1) * stride < nvec; i += U * stride) {
    D2 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT) {
        r[u].x = __builtin_nontemporal_load(&v[i + u * stride].x);
        r[u].y = __builtin_nontemporal_load(&v[i + u * stride].y);
      } else {
        r[u] = v[i + u * stride];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] += r[u].x * r[u].x + r[u].y * r[u].y;
  }
  for (; i < nvec; i += stride) acc[0] += v[i].x * v[i].x + v[i].y * v[i].y;
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u) s += acc[u];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  __shared__ double w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// y = x*x over f64x2 vectors; LNT / SNT: non-temporal loads / stores
template <bool LNT, bool SNT>
__global__ __launch_bounds__(256) void sqcopy(const double* __restrict__ a, double* __restrict__ b, int64_t n) {
  const int64_t nvec = n / 2;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const u32x4* src = reinterpret_cast<const u32x4*>(a);
  u32x4* dst = reinterpret_cast<u32x4*>(b);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += stride) {
    u32x4 r = LNT ? __builtin_nontemporal_load(src + i) : src[i];
    D2 d = *reinterpret_cast<D2*>(&r);
    d.x *= d.x;
    d.y *= d.y;
    u32x4 w = *reinterpret_cast<u32x4*>(&d);
    if (SNT) __builtin_nontemporal_store(w, dst + i);
    else dst[i] = w;
  }
}

template <bool LNT, bool SNT>
void run_copy(const double* a, double* b, int64_t n, int grid, hipEvent_t s, hipEvent_t e) {
  float best = 1e9f;
  for (int rep = 0; rep < 20; ++rep) {
    hipEventRecord(s);
    sqcopy<LNT, SNT><<<grid, 256>>>(a, b, n);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    if (rep > 2 && ms < best) best = ms;
  }
  printf("{\"square_copy\": 1, \"ld_nt\": %d, \"st_nt\": %d, \"grid\": %d, \"best_us\": %.2f, \"TBps\": %.3f}\n", (int)LNT,
         (int)SNT, grid, best * 1e3, n * 16.0 / (best * 1e-3) / 1e12);
}

__global__ void fill(double* a, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    a[i] = (double)((i * 2654435761ull) % 1000003) / 1000003.0;
}

template <int U, bool NT>
void run(const double* a, int64_t n, double* part, int grid, hipEvent_t s, hipEvent_t e) {
  float best = 1e9f;
  for (int rep = 0; rep < 20; ++rep) {
    hipEventRecord(s);
    sqsum<U, NT><<<grid, 256>>>(a, n, part);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    if (rep > 2 && ms < best) best = ms;
  }
  printf("{\"U\": %d, \"nt\": %d, \"grid\": %d, \"best_us\": %.2f, \"TBps\": %.3f}\n", U, (int)NT, grid, best * 1e3,
         n * 8.0 / (best * 1e-3) / 1e12);
}

int main() {
  const int64_t n = 100000000;
  double *a, *part;
  if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&part, 65536 * 8) != hipSuccess) return 1;
  fill<<<4096, 256>>>(a, n);
  hipDeviceSynchronize();
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  double* b;
  if (hipMalloc(&b, n * 8) != hipSuccess) return 1;
  for (int grid : {8192, 16384, 32768}) {
    run_copy<false, false>(a, b, n, grid, s, e);
    run_copy<true, false>(a, b, n, grid, s, e);
    run_copy<false, true>(a, b, n, grid, s, e);
    run_copy<true, true>(a, b, n, grid, s, e);
  }
  for (int grid : {8192, 16384}) {
    run<16, true>(a, n, part, grid, s, e);
  }
  for (int grid : {1024, 2048, 4096, 8192}) {
    run<4, false>(a, n, part, grid, s, e);
    run<8, false>(a, n, part, grid, s, e);
    run<4, true>(a, n, part, grid, s, e);
    run<8, true>(a, n, part, grid, s, e);
  }
  return 0;
}
