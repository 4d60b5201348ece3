// stream_beside.hip — diagnostic: an HBM read-modify-write stream on a
// CU-masked stream, to measure the persistent chain beside a flush-like
// stream ("chain beside the flush").  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/dbg/libstream_beside.so tools/dbg/stream_beside.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>
#include <vector>

typedef double dbl2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void rmw_kernel(dbl2* __restrict__ a, int64_t n, double s) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    dbl2 x = __builtin_nontemporal_load(a + i);
    x.x = x.x * s;
    x.y = x.y * s;
    __builtin_nontemporal_store(x, a + i);
  }
}

static hipStream_t g_stream = nullptr;
static dbl2* g_buf = nullptr;
static int64_t g_n = 0;
static int g_grid = 0;

extern "C" {
// every `every`-th CU is left out of the stream's mask (0: all CUs)
int sb_init(int every, int64_t bytes) {
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return -1;
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  int on = 0;
  for (int c = 0; c < ncu; ++c)
    if (every <= 0 || c % every != 0) {
      mask[c / 32] |= 1u << (c % 32);
      ++on;
    }
  if (hipExtStreamCreateWithCUMask(&g_stream, (uint32_t)mask.size(), mask.data()) != hipSuccess)
    return -2;
  g_n = bytes / 16;
  if (hipMalloc(&g_buf, g_n * 16) != hipSuccess) return -3;
  if (hipMemset(g_buf, 0, g_n * 16) != hipSuccess) return -4;
  g_grid = on * 8;
  return on;
}
int sb_run(int iters) {
  for (int k = 0; k < iters; ++k)
    hipLaunchKernelGGL(rmw_kernel, dim3(g_grid), dim3(256), 0, g_stream, g_buf, g_n, 1.0);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// milliseconds of `iters` stream passes alone (events)
double sb_time(int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, g_stream);
  sb_run(iters);
  hipEventRecord(b, g_stream);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms;
}
int sb_sync() { return hipStreamSynchronize(g_stream) == hipSuccess ? 0 : -1; }
int sb_query() { return hipStreamQuery(g_stream) == hipSuccess ? 1 : 0; }  // 1: idle
}
