// Checks wave_min_dpp against wave_min (ds_bpermute) on random keys with ties.
#include <cstdio>
#include <cstdlib>
#include "../../simplex-solver_amd/csrc/spx_kernels.hpp"
using namespace spx;
__global__ void kcheck(const double* v, const int64_t* t, const int64_t* r, int64_t* out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  KeyR a{v[i], t[i], r[i]}, b = a;
  wave_min(a);
  wave_min_dpp(b);
  out[3 * i + 0] = (a.v == b.v);
  out[3 * i + 1] = (a.t == b.t);
  out[3 * i + 2] = (a.row == b.row);
}
int main() {
  const int W = 4096, n = W * 64;
  double* hv = (double*)malloc(8 * n); int64_t* ht = (int64_t*)malloc(8 * n); int64_t* hr = (int64_t*)malloc(8 * n);
  srand(7);
  for (int i = 0; i < n; ++i) {
    hv[i] = (rand() % 5 == 0) ? __builtin_inf() : (double)(rand() % 7);  // many ties
    ht[i] = rand() % 100000; hr[i] = i;
  }
  double* dv; int64_t *dt, *dr, *dout;
  hipMalloc(&dv, 8 * n); hipMalloc(&dt, 8 * n); hipMalloc(&dr, 8 * n); hipMalloc(&dout, 24 * n);
  hipMemcpy(dv, hv, 8 * n, hipMemcpyHostToDevice); hipMemcpy(dt, ht, 8 * n, hipMemcpyHostToDevice);
  hipMemcpy(dr, hr, 8 * n, hipMemcpyHostToDevice);
  kcheck<<<W, 64>>>(dv, dt, dr, dout);
  int64_t* ho = (int64_t*)malloc(24 * n);
  hipMemcpy(ho, dout, 24 * n, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < 3 * n; ++i) bad += (ho[i] != 1);
  printf("dpp_check: %ld mismatching components of %d\n", bad, 3 * n);
  return bad != 0;
}
