#include <hip/hip_runtime.h>
extern "C" __global__ void fill_k(float* p, float v, long n){ long i = blockIdx.x*(long)blockDim.x+threadIdx.x; if(i<n) p[i]=v; }
extern "C" int probe_fill(float* p, float v, long n, hipStream_t s){ hipLaunchKernelGGL(fill_k, dim3((n+255)/256), dim3(256), 0, s, p, v, n); return (int)hipGetLastError(); }
