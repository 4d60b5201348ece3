// hbm_ceiling.hip — STREAM-style HBM ceiling on MI355X for the access shapes of
// the elimination kernel (16-B lanes, fp64): read-only, copy, and in-place
// read-modify-write x = x - a*b, each with plain and non-temporal hints.
// Prints one JSON line per variant: GB/s = (bytes read + bytes written) / time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <bool NT>
__global__ __launch_bounds__(256) void rmw(dbl2* __restrict__ x, size_t n2, double a, double b) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
    dbl2 v = NT ? __builtin_nontemporal_load(x + i) : x[i];
    v.x = v.x - a * b;
    v.y = v.y - a * b;
    if (NT) __builtin_nontemporal_store(v, x + i); else x[i] = v;
  }
}
template <bool NT>
__global__ __launch_bounds__(256) void copy(const dbl2* __restrict__ x, dbl2* __restrict__ y,
                                            size_t n2) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
    dbl2 v = NT ? __builtin_nontemporal_load(x + i) : x[i];
    if (NT) __builtin_nontemporal_store(v, y + i); else y[i] = v;
  }
}
__global__ __launch_bounds__(256) void readk(const dbl2* __restrict__ x, size_t n2, double* out) {
  double s = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
    dbl2 v = x[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}

#define CK(x) do { hipError_t e = (x); if (e) { printf("err %s\n", hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const size_t bytes = size_t(1) << 30;  // 1 GiB per buffer (> 256 MiB Infinity Cache)
  const size_t n2 = bytes / 16;
  dbl2 *x, *y;
  double* out;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(x, 0, bytes));
  CK(hipMemset(y, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grids[] = {1024, 2048, 4096, 8192};
  for (int rep = 0; rep < 2; ++rep)
    for (int g : grids)
      for (int v = 0; v < 5; ++v) {
        float best = 1e30f;
        for (int it = 0; it < 6; ++it) {
          CK(hipEventRecord(e0));
          switch (v) {
            case 0: rmw<false><<<g, 256>>>(x, n2, 1.0, 0.0); break;
            case 1: rmw<true><<<g, 256>>>(x, n2, 1.0, 0.0); break;
            case 2: copy<false><<<g, 256>>>(x, y, n2); break;
            case 3: copy<true><<<g, 256>>>(x, y, n2); break;
            case 4: readk<<<g, 256>>>(x, n2, out); break;
          }
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (it > 0 && ms < best) best = ms;
        }
        const char* names[] = {"rmw", "rmw_nt", "copy", "copy_nt", "read"};
        const double moved = (v == 4) ? bytes : 2.0 * bytes;
        if (rep == 1)
          printf("{\"kernel\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", names[v], g,
                 best, moved / (best * 1e-3) / 1e9);
      }
  return 0;
}
