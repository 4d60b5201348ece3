// Latency floor probe for the per-pivot critical path (windowed
// elimination): what a dependent kernel boundary costs inside a hipGraph, and
// what a grid-wide barrier inside one persistent kernel costs instead.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/latency_probe tools/latency_probe.hip
//   tools/latency_probe
//
// Every spin loop has a wall-clock exit (s_memrealtime, 100 MHz), so a
// non-resident grid ends with an error count instead of hanging the GPU.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

__global__ void empty_kernel() {}

// each block reads a value the previous launch wrote (a dependent chain)
__global__ void chain_kernel(double* buf, int n) {
  __shared__ double s;
  if (threadIdx.x == 0) s = buf[(blockIdx.x + 1) % n];
  __syncthreads();
  if (threadIdx.x == 0) buf[blockIdx.x] = s + 1.0;
}

__device__ __forceinline__ unsigned long long now_ticks() {
  return __builtin_amdgcn_s_memrealtime();
}

// persistent kernel: `rounds` grid barriers; between barriers every block
// publishes one value and reads another block's value from the last round.
__global__ void barrier_kernel(unsigned* ctr, double* vals, int rounds, int* errs) {
  const unsigned nb = gridDim.x;
  for (int k = 1; k <= rounds; ++k) {
    if (threadIdx.x == 0) vals[(k & 1) * nb + blockIdx.x] = (double)(k * 1000 + blockIdx.x);
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)k * nb;
      const unsigned long long t0 = now_ticks();
      while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (now_ticks() - t0 > 5000000ull) {  // 50 ms
          atomicAdd(errs, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const unsigned other = (blockIdx.x + 1) % nb;
      if (vals[(k & 1) * nb + other] != (double)(k * 1000 + other)) atomicAdd(errs + 1, 1);
    }
    __syncthreads();
  }
}

int main() {
  const int NK = 1000;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  double* buf;
  CK(hipMalloc(&buf, 1 << 20));
  CK(hipMemset(buf, 0, 1 << 20));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms;
  for (int blocks : {1, 16, 64, 256}) {
    for (int kind = 0; kind < 2; ++kind) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < NK; ++i) {
        if (kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, s);
        else hipLaunchKernelGGL(chain_kernel, dim3(blocks), dim3(256), 0, s, buf, blocks);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("{\"probe\": \"%s_kernel_in_graph\", \"blocks\": %d, \"us_per_kernel\": %.3f}\n",
                  kind ? "dependent_chain" : "empty", blocks, 1e3 * ms / NK);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  unsigned* ctr;
  int* errs;
  double* vals;
  CK(hipMalloc(&ctr, sizeof(unsigned)));
  CK(hipMalloc(&errs, 2 * sizeof(int)));
  CK(hipMalloc(&vals, 2 * 1024 * sizeof(double)));
  for (int blocks : {16, 32, 64, 128, 256}) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(ctr, 0, sizeof(unsigned)));
      CK(hipMemset(errs, 0, 2 * sizeof(int)));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, s));
      hipLaunchKernelGGL(barrier_kernel, dim3(blocks), dim3(256), 0, s, ctr, vals, NK, errs);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      int he[2];
      CK(hipMemcpy(he, errs, sizeof(he), hipMemcpyDeviceToHost));
      if (rep)
        std::printf("{\"probe\": \"grid_barrier\", \"blocks\": %d, \"us_per_barrier\": %.3f, "
                    "\"timeouts\": %d, \"stale_reads\": %d}\n",
                    blocks, 1e3 * ms / NK, he[0], he[1]);
    }
  }
  return 0;
}
