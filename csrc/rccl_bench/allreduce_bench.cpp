// bee-rccl-bench: native RCCL all-reduce sweep over the GPUs of one node
// (BASELINE config 5 / SURVEY.md §2.2), independent of torch.
//
// One process drives every visible GPU: ncclCommInitAll + one HIP stream per
// device, group-launched ncclAllReduce per message size.  Reports per size:
// time, algbw = bytes / t and busbw = algbw * 2(n-1)/n — the number to hold
// against the per-GPU xGMI budget (7 links x ~153 GB/s per direction on
// MI355X; a single ring uses one link per hop, RCCL spreads channels over
// links).  Every size is checked on every GPU (its first and last 2048
// elements against n(n+1)/2), and a row says "checked": true only then; the
// exit status is non-zero if any check failed.
//
//   bee-rccl-bench [--gpus N] [--min BYTES] [--max BYTES] [--iters K] [--dtype f32|bf16]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HIPCHECK(x)                                                                            \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
      exit(2);                                                                                 \
    }                                                                                          \
  } while (0)
#define NCCLCHECK(x)                                                                           \
  do {                                                                                         \
    ncclResult_t r_ = (x);                                                                     \
    if (r_ != ncclSuccess) {                                                                   \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      exit(3);                                                                                 \
    }                                                                                          \
  } while (0)

template <typename T>
__global__ void fill_kernel(T* p, size_t n, T v) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) p[i] = v;
}

// bf16 bits of a small integer-valued float (exact for the checks here)
static uint16_t to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}
static float from_bf16(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static int64_t parse_size(const char* s) {
  char* end = nullptr;
  double v = strtod(s, &end);
  if (end && (*end == 'K' || *end == 'k')) v *= 1024;
  if (end && (*end == 'M' || *end == 'm')) v *= 1024 * 1024;
  if (end && (*end == 'G' || *end == 'g')) v *= 1024.0 * 1024 * 1024;
  return (int64_t)v;
}

int main(int argc, char** argv) {
  int ngpus = 0;
  HIPCHECK(hipGetDeviceCount(&ngpus));
  int64_t min_bytes = 1 << 10, max_bytes = 1LL << 30;
  int iters = 20;
  std::string dtype = "f32";
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--gpus" && i + 1 < argc) ngpus = std::min(ngpus, atoi(argv[++i]));
    else if (a == "--min" && i + 1 < argc) min_bytes = parse_size(argv[++i]);
    else if (a == "--max" && i + 1 < argc) max_bytes = parse_size(argv[++i]);
    else if (a == "--iters" && i + 1 < argc) iters = atoi(argv[++i]);
    else if (a == "--dtype" && i + 1 < argc) dtype = argv[++i];
    else {
      fprintf(stderr, "usage: bee-rccl-bench [--gpus N] [--min BYTES] [--max BYTES] [--iters K] [--dtype f32|bf16]\n");
      return 1;
    }
  }
  if (dtype != "f32" && dtype != "bf16") {
    fprintf(stderr, "--dtype must be f32 or bf16\n");
    return 1;
  }
  const bool bf16 = dtype == "bf16";
  const size_t es = bf16 ? 2 : 4;
  const ncclDataType_t nt = bf16 ? ncclBfloat16 : ncclFloat;
  if (ngpus < 1) {
    fprintf(stderr, "no GPUs\n");
    return 1;
  }
  std::vector<int> devs(ngpus);
  for (int i = 0; i < ngpus; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(ngpus);
  NCCLCHECK(ncclCommInitAll(comms.data(), ngpus, devs.data()));
  std::vector<hipStream_t> streams(ngpus);
  std::vector<void*> buf(ngpus);
  const size_t max_count = (size_t)(max_bytes / es);
  for (int i = 0; i < ngpus; ++i) {
    HIPCHECK(hipSetDevice(i));
    HIPCHECK(hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking));
    HIPCHECK(hipMalloc(&buf[i], max_count * es));
  }
  printf("{\"tool\": \"bee-rccl-bench\", \"gpus\": %d, \"dtype\": \"%s\", \"rccl_version\": %d}\n", ngpus,
         dtype.c_str(), NCCL_VERSION_CODE);
  bool all_ok = true;
  for (int64_t bytes = min_bytes; bytes <= max_bytes; bytes *= 2) {
    const size_t count = (size_t)(bytes / es);
    for (int i = 0; i < ngpus; ++i) {
      HIPCHECK(hipSetDevice(i));
      if (bf16)
        hipLaunchKernelGGL(fill_kernel<uint16_t>, dim3(1024), dim3(256), 0, streams[i], (uint16_t*)buf[i], count,
                           to_bf16((float)(i + 1)));
      else
        hipLaunchKernelGGL(fill_kernel<float>, dim3(1024), dim3(256), 0, streams[i], (float*)buf[i], count,
                           (float)(i + 1));
    }
    auto run = [&](int k) {
      for (int it = 0; it < k; ++it) {
        NCCLCHECK(ncclGroupStart());
        for (int i = 0; i < ngpus; ++i)
          NCCLCHECK(ncclAllReduce(buf[i], buf[i], count, nt, ncclSum, comms[i], streams[i]));
        NCCLCHECK(ncclGroupEnd());
      }
      for (int i = 0; i < ngpus; ++i) {
        HIPCHECK(hipSetDevice(i));
        HIPCHECK(hipStreamSynchronize(streams[i]));
      }
    };
    run(1);  // correctness: every element = n(n+1)/2, on every GPU
    bool ok = true;
    {
      const size_t nh = std::min<size_t>(count, 2048);
      std::vector<char> host(nh * es);
      const float want = ngpus * (ngpus + 1) / 2.0f;
      for (int g = 0; g < ngpus && ok; ++g) {
        HIPCHECK(hipSetDevice(g));
        // the head and the tail of the buffer (a channel that drops its last
        // chunk shows at the end)
        for (size_t start : {(size_t)0, count - nh}) {
          HIPCHECK(hipMemcpy(host.data(), (char*)buf[g] + start * es, host.size(), hipMemcpyDeviceToHost));
          for (size_t k = 0; k < nh; ++k) {
            float v;
            if (bf16) {
              uint16_t b;
              memcpy(&b, host.data() + k * 2, 2);
              v = from_bf16(b);
            } else {
              memcpy(&v, host.data() + k * 4, 4);
            }
            ok = ok && v == want;
          }
        }
      }
      all_ok = all_ok && ok;
    }
    run(2);  // warm
    auto t0 = std::chrono::steady_clock::now();
    run(iters);
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
    double algbw = bytes / s / 1e9;
    double busbw = algbw * (ngpus > 1 ? 2.0 * (ngpus - 1) / ngpus : 1.0);
    printf("{\"bytes\": %lld, \"us\": %.2f, \"algbw_GBps\": %.2f, \"busbw_GBps\": %.2f, \"checked\": %s}\n",
           (long long)bytes, s * 1e6, algbw, busbw, ok ? "true" : "false");
    fflush(stdout);
  }
  for (int i = 0; i < ngpus; ++i) {
    HIPCHECK(hipSetDevice(i));
    HIPCHECK(hipFree(buf[i]));
    ncclCommDestroy(comms[i]);
  }
  return all_ok ? 0 : 4;
}
