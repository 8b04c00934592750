// bee-rccl-bench: native RCCL all-reduce sweep over the GPUs of one node
// (BASELINE config 5 / SURVEY.md §2.2), independent of torch.
//
// One process drives every visible GPU: ncclCommInitAll + one HIP stream per
// device, group-launched ncclAllReduce per message size.  Reports per size:
// time, algbw = bytes / t and busbw = algbw * 2(n-1)/n — the number to hold
// against the per-GPU xGMI budget (7 links x ~153 GB/s per direction on
// MI355X; a single ring uses one link per hop, RCCL spreads channels over
// links).  Correctness is checked on the first and last size.
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

__global__ void fill_kernel(float* p, size_t n, float v) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) p[i] = v;
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
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--gpus" && i + 1 < argc) ngpus = std::min(ngpus, atoi(argv[++i]));
    else if (a == "--min" && i + 1 < argc) min_bytes = parse_size(argv[++i]);
    else if (a == "--max" && i + 1 < argc) max_bytes = parse_size(argv[++i]);
    else if (a == "--iters" && i + 1 < argc) iters = atoi(argv[++i]);
  }
  if (ngpus < 1) {
    fprintf(stderr, "no GPUs\n");
    return 1;
  }
  std::vector<int> devs(ngpus);
  for (int i = 0; i < ngpus; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(ngpus);
  NCCLCHECK(ncclCommInitAll(comms.data(), ngpus, devs.data()));
  std::vector<hipStream_t> streams(ngpus);
  std::vector<float*> buf(ngpus);
  const size_t max_count = (size_t)(max_bytes / 4);
  for (int i = 0; i < ngpus; ++i) {
    HIPCHECK(hipSetDevice(i));
    HIPCHECK(hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking));
    HIPCHECK(hipMalloc(&buf[i], max_count * sizeof(float)));
  }
  printf("{\"tool\": \"bee-rccl-bench\", \"gpus\": %d, \"rccl_version\": %d}\n", ngpus, NCCL_VERSION_CODE);
  bool all_ok = true;
  for (int64_t bytes = min_bytes; bytes <= max_bytes; bytes *= 2) {
    const size_t count = (size_t)(bytes / 4);
    for (int i = 0; i < ngpus; ++i) {
      HIPCHECK(hipSetDevice(i));
      hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, streams[i], buf[i], count, (float)(i + 1));
    }
    auto run = [&](int k) {
      for (int it = 0; it < k; ++it) {
        NCCLCHECK(ncclGroupStart());
        for (int i = 0; i < ngpus; ++i)
          NCCLCHECK(ncclAllReduce(buf[i], buf[i], count, ncclFloat, ncclSum, comms[i], streams[i]));
        NCCLCHECK(ncclGroupEnd());
      }
      for (int i = 0; i < ngpus; ++i) {
        HIPCHECK(hipSetDevice(i));
        HIPCHECK(hipStreamSynchronize(streams[i]));
      }
    };
    run(1);  // correctness: every element = n(n+1)/2
    bool ok = true;
    if (bytes == min_bytes || bytes * 2 > max_bytes) {
      std::vector<float> host(std::min<size_t>(count, 4096));
      HIPCHECK(hipSetDevice(ngpus - 1));
      HIPCHECK(hipMemcpy(host.data(), buf[ngpus - 1], host.size() * 4, hipMemcpyDeviceToHost));
      const float want = ngpus * (ngpus + 1) / 2.0f;
      for (float v : host) ok = ok && v == want;
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
