// Elementwise kernels (square, unary math, binary arithmetic, casts).
//
// HBM-bound: every lane moves 16 bytes per access (f64x2 / f32x4 / bf16x8,
// Guideline 13), non-temporal for arrays past the Infinity Cache
// (bk_common.hpp ld16/st16), grid-stride over <= 64 blocks per CU.  bf16 math runs in f32
// and rounds once on store.  `numpy.square` of the benchmark payload
// (`examples/benchmark-numpy.py:21`) is kUnarySquare on f64.
#include "bk_common.hpp"

namespace bk {

enum UnaryOp : int {
  kUnarySquare = 0, kUnaryAbs, kUnaryNeg, kUnarySqrt, kUnaryExp, kUnaryLog, kUnaryRelu,
  kUnarySin, kUnaryCos, kUnaryTanh, kUnarySigmoid, kUnaryCopy, kUnaryCount
};
enum BinaryOp : int { kBinAdd = 0, kBinSub, kBinMul, kBinDiv, kBinMax, kBinMin, kBinPow, kBinCount };

template <typename T> struct Elem;  // storage <-> compute type
template <> struct Elem<float> {
  using C = float;
  __device__ static C load(float v) { return v; }
  __device__ static float store(C v) { return v; }
};
template <> struct Elem<double> {
  using C = double;
  __device__ static C load(double v) { return v; }
  __device__ static double store(C v) { return v; }
};
template <> struct Elem<uint16_t> {  // bf16 bits
  using C = float;
  __device__ static C load(uint16_t v) { return bf16_bits_to_float(v); }
  __device__ static uint16_t store(C v) { return float_to_bf16_bits(v); }
};

template <int OP, typename C>
__device__ __forceinline__ C unary(C x) {
  if constexpr (OP == kUnarySquare) return x * x;
  else if constexpr (OP == kUnaryAbs) return x < C(0) ? -x : x;
  else if constexpr (OP == kUnaryNeg) return -x;
  else if constexpr (OP == kUnarySqrt) return sqrt(x);
  else if constexpr (OP == kUnaryExp) return exp(x);
  else if constexpr (OP == kUnaryLog) return log(x);
  else if constexpr (OP == kUnaryRelu) return x > C(0) ? x : C(0);
  else if constexpr (OP == kUnarySin) return sin(x);
  else if constexpr (OP == kUnaryCos) return cos(x);
  else if constexpr (OP == kUnaryTanh) return tanh(x);
  else if constexpr (OP == kUnarySigmoid) return C(1) / (C(1) + exp(-x));
  else return x;
}

template <int OP, typename C>
__device__ __forceinline__ C binary(C a, C b) {
  if constexpr (OP == kBinAdd) return a + b;
  else if constexpr (OP == kBinSub) return a - b;
  else if constexpr (OP == kBinMul) return a * b;
  else if constexpr (OP == kBinDiv) return a / b;
  // numpy.maximum / minimum: NaN in either operand gives NaN
  else if constexpr (OP == kBinMax) return (a > b || a != a) ? a : b;
  else if constexpr (OP == kBinMin) return (a < b || a != a) ? a : b;
  else return pow(a, b);
}

template <typename T>
struct alignas(16) Vec {
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};

constexpr int kEwUnroll = 4;  // 16-B loads in flight per lane before the first store

template <typename T, int OP, bool NT>
__global__ __launch_bounds__(256) void unary_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n) {
  using E = Elem<T>;
  using V = Vec<T>;
  constexpr int N = V::N, U = kEwUnroll;
  const int64_t nvec = n / N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const V* xv = reinterpret_cast<const V*>(x);
  V* yv = reinterpret_cast<V*>(y);
  // block-contiguous chunks of U*256 vectors: each load instruction of a wave
  // covers 1 KiB contiguous and a block's U instructions one 16 KiB span
  const int64_t chunk = (int64_t)U * blockDim.x;
  const int64_t nfull = nvec / chunk;
  for (int64_t cb = blockIdx.x; cb < nfull; cb += gridDim.x) {
    const int64_t base = cb * chunk + threadIdx.x;
    V a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld16<NT>(xv + base + u * blockDim.x);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < N; ++j) a[u].v[j] = E::store(unary<OP>(E::load(a[u].v[j])));
#pragma unroll
    for (int u = 0; u < U; ++u) st16<NT>(yv + base + u * blockDim.x, a[u]);
  }
  for (int64_t i = nfull * chunk + tid; i < nvec; i += stride) {
    V a = xv[i];
#pragma unroll
    for (int j = 0; j < N; ++j) a.v[j] = E::store(unary<OP>(E::load(a.v[j])));
    yv[i] = a;
  }
  for (int64_t k = nvec * N + tid; k < n; k += stride) y[k] = E::store(unary<OP>(E::load(x[k])));
}

// y = op(a, b) with b an array (B_SCALAR=false) or a scalar (B_SCALAR=true);
// REVERSED swaps the operands for scalar ops (s - x, s / x, ...).
template <typename T, int OP, bool B_SCALAR, bool REVERSED, bool NT>
__global__ __launch_bounds__(256) void binary_kernel(const T* __restrict__ a, const T* __restrict__ b, double s,
                                                     T* __restrict__ y, int64_t n) {
  using E = Elem<T>;
  using C = typename E::C;
  using V = Vec<T>;
  constexpr int N = V::N;
  constexpr int U = kEwUnroll;
  const C sc = (C)s;
  const int64_t nvec = n / N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const V* av = reinterpret_cast<const V*>(a);
  const V* bv = reinterpret_cast<const V*>(b);
  V* yv = reinterpret_cast<V*>(y);
  auto apply = [&](V& va, const V& vb) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const C lhs = E::load(va.v[j]);
      const C rhs = B_SCALAR ? sc : E::load(vb.v[j]);
      va.v[j] = E::store(REVERSED ? binary<OP>(rhs, lhs) : binary<OP>(lhs, rhs));
    }
  };
  const int64_t chunk = (int64_t)U * blockDim.x;
  const int64_t nfull = nvec / chunk;
  for (int64_t cb = blockIdx.x; cb < nfull; cb += gridDim.x) {
    const int64_t base = cb * chunk + threadIdx.x;
    V va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = ld16<NT>(av + base + u * blockDim.x);
      if constexpr (!B_SCALAR) vb[u] = ld16<NT>(bv + base + u * blockDim.x);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) apply(va[u], vb[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) st16<NT>(yv + base + u * blockDim.x, va[u]);
  }
  for (int64_t i = nfull * chunk + tid; i < nvec; i += stride) {
    V va = av[i], vb;
    if constexpr (!B_SCALAR) vb = bv[i];
    apply(va, vb);
    yv[i] = va;
  }
  for (int64_t k = nvec * N + tid; k < n; k += stride) {
    const C lhs = E::load(a[k]);
    const C rhs = B_SCALAR ? sc : E::load(b[k]);
    y[k] = E::store(REVERSED ? binary<OP>(rhs, lhs) : binary<OP>(lhs, rhs));
  }
}

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if constexpr (std::is_same<TI, double>::value && std::is_same<TO, uint16_t>::value)
      y[i] = double_to_bf16_bits(x[i]);
    else
      y[i] = Elem<TO>::store((typename Elem<TO>::C)Elem<TI>::load(x[i]));
  }
}

__global__ __launch_bounds__(256) void fill_kernel(uint8_t* __restrict__ y, int64_t nbytes, uint64_t pattern,
                                                   int pattern_bytes) {
  // pattern_bytes in {1,2,4,8}; 16-B stores for the bulk.
  uint64_t p = pattern;
  if (pattern_bytes == 1) p = (p & 0xff) * 0x0101010101010101ull;
  if (pattern_bytes == 2) p = (p & 0xffff) * 0x0001000100010001ull;
  if (pattern_bytes == 4) p = (p & 0xffffffffull) | ((p & 0xffffffffull) << 32);
  const uint4 v = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)p, (uint32_t)(p >> 32));
  const int64_t nvec = nbytes / 16;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = tid; i < nvec; i += stride) reinterpret_cast<uint4*>(y)[i] = v;
  for (int64_t i = nvec * 16 + tid; i < nbytes; i += stride) y[i] = (uint8_t)(p >> (8 * (i % 8)));
}

// ---- host dispatch ---------------------------------------------------------
template <typename T, int OP>
int launch_unary_t(const void* x, void* y, int64_t n, hipStream_t s) {
  const unsigned g = stream_grid((n + Vec<T>::N - 1) / Vec<T>::N, 256);
  if (stream_nt(n * (int64_t)sizeof(T))) unary_kernel<T, OP, true><<<g, 256, 0, s>>>((const T*)x, (T*)y, n);
  else unary_kernel<T, OP, false><<<g, 256, 0, s>>>((const T*)x, (T*)y, n);
  return launch_status();
}

template <typename T, int... OPS>
int dispatch_unary(int op, const void* x, void* y, int64_t n, hipStream_t s, std::integer_sequence<int, OPS...>) {
  int rc = kBadArgument;
  ((op == OPS ? (rc = launch_unary_t<T, OPS>(x, y, n, s), 0) : 0), ...);
  return rc;
}

template <typename T, int OP, bool BS, bool REV>
int launch_binary_t(const void* a, const void* b, double sc, void* y, int64_t n, hipStream_t s) {
  const unsigned g = stream_grid((n + Vec<T>::N - 1) / Vec<T>::N, 256);
  if (stream_nt(n * (int64_t)sizeof(T)))
    binary_kernel<T, OP, BS, REV, true><<<g, 256, 0, s>>>((const T*)a, (const T*)b, sc, (T*)y, n);
  else
    binary_kernel<T, OP, BS, REV, false><<<g, 256, 0, s>>>((const T*)a, (const T*)b, sc, (T*)y, n);
  return launch_status();
}

template <typename T, int... OPS>
int dispatch_binary(int op, int mode, const void* a, const void* b, double sc, void* y, int64_t n, hipStream_t s,
                    std::integer_sequence<int, OPS...>) {
  int rc = kBadArgument;
  auto one = [&](auto opc) {
    constexpr int OP = decltype(opc)::value;
    if (mode == 0) rc = launch_binary_t<T, OP, false, false>(a, b, sc, y, n, s);
    else if (mode == 1) rc = launch_binary_t<T, OP, true, false>(a, b, sc, y, n, s);
    else rc = launch_binary_t<T, OP, true, true>(a, b, sc, y, n, s);
  };
  ((op == OPS ? (one(std::integral_constant<int, OPS>{}), 0) : 0), ...);
  return rc;
}

}  // namespace bk

using namespace bk;

BK_API int bk_unary(int op, int dtype, const void* x, void* y, int64_t n, hipStream_t stream) {
  if (!x || !y || n < 0 || op < 0 || op >= kUnaryCount) return kBadArgument;
  if (n == 0) return kOk;
  using Ops = std::make_integer_sequence<int, kUnaryCount>;
  switch (dtype) {
    case kF32: return dispatch_unary<float>(op, x, y, n, stream, Ops{});
    case kF64: return dispatch_unary<double>(op, x, y, n, stream, Ops{});
    case kBF16: return dispatch_unary<uint16_t>(op, x, y, n, stream, Ops{});
  }
  return kBadArgument;
}

// mode: 0 = array (op) array, 1 = array (op) scalar, 2 = scalar (op) array
BK_API int bk_binary(int op, int dtype, int mode, const void* a, const void* b, double scalar, void* y, int64_t n,
                     hipStream_t stream) {
  if (!a || !y || n < 0 || op < 0 || op >= kBinCount || mode < 0 || mode > 2 || (mode == 0 && !b))
    return kBadArgument;
  if (n == 0) return kOk;
  using Ops = std::make_integer_sequence<int, kBinCount>;
  switch (dtype) {
    case kF32: return dispatch_binary<float>(op, mode, a, b, scalar, y, n, stream, Ops{});
    case kF64: return dispatch_binary<double>(op, mode, a, b, scalar, y, n, stream, Ops{});
    case kBF16: return dispatch_binary<uint16_t>(op, mode, a, b, scalar, y, n, stream, Ops{});
  }
  return kBadArgument;
}

BK_API int bk_cast(int src_dtype, int dst_dtype, const void* x, void* y, int64_t n, hipStream_t stream) {
  if (!x || !y || n < 0) return kBadArgument;
  if (n == 0) return kOk;
  const unsigned g = stream_grid(n, 256);
#define BK_CAST(TI, TO) cast_kernel<TI, TO><<<g, 256, 0, stream>>>((const TI*)x, (TO*)y, n)
  if (src_dtype == kF32 && dst_dtype == kBF16) BK_CAST(float, uint16_t);
  else if (src_dtype == kBF16 && dst_dtype == kF32) BK_CAST(uint16_t, float);
  else if (src_dtype == kF64 && dst_dtype == kF32) BK_CAST(double, float);
  else if (src_dtype == kF32 && dst_dtype == kF64) BK_CAST(float, double);
  else if (src_dtype == kF64 && dst_dtype == kBF16) BK_CAST(double, uint16_t);
  else if (src_dtype == kBF16 && dst_dtype == kF64) BK_CAST(uint16_t, double);
  else return kBadArgument;
#undef BK_CAST
  return launch_status();
}

BK_API int bk_fill(void* y, int64_t nbytes, uint64_t pattern, int pattern_bytes, hipStream_t stream) {
  if (!y || nbytes < 0 || !(pattern_bytes == 1 || pattern_bytes == 2 || pattern_bytes == 4 || pattern_bytes == 8))
    return kBadArgument;
  if (nbytes == 0) return kOk;
  fill_kernel<<<stream_grid((nbytes + 15) / 16, 256), 256, 0, stream>>>((uint8_t*)y, nbytes, pattern, pattern_bytes);
  return launch_status();
}
