// chain_probe.hip — latency of an in-launch all-to-all exchange (diagnostic).
//
// A persistent grid of B blocks repeats, `iters` times: every block publishes
// G tagged 8-byte granules {tag, value} (one sc1 store each), one wave per
// block polls all B*G granules (sc1 loads) until every tag matches, reduces
// the values, and issues one dependent load from a 1 GiB buffer at an address
// derived from the reduced value (the pivot chain's dependent HBM round trip).
// Reports us per exchange for B in {32, 64, 128, 256}, G in {3, 8}: the price
// of one pivot-chain phase without a kernel boundary.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ __launch_bounds__(256) void chain(unsigned long long* rec_, int G, const double* big,
                                             size_t nbig, int iters, unsigned* tmo_, double* out,
                                             int dep) {
  gu64* rec = (gu64*)rec_;
  gu32* tmo = (gu32*)tmo_;
  __shared__ unsigned bval;
  __shared__ char pad_lds[96 * 1024];  // one block per CU
  const int lane = threadIdx.x & 63;
  const int B = gridDim.x;
  const int n = B * G;
  unsigned v = blockIdx.x;
  double acc = 0.0;
  if (threadIdx.x == 0) pad_lds[blockIdx.x & 1023] = 0;
  for (int it = 0; it < iters; ++it) {
    const unsigned tag = (unsigned)it + 1u;
    // granules double-buffered by parity: a block can be at most one exchange
    // ahead of the slowest reader
    gu64* rb = rec + (size_t)(it & 1) * 256 * 16;
    if (threadIdx.x < G)
      __hip_atomic_store(rb + (size_t)blockIdx.x * G + threadIdx.x,
                         ((unsigned long long)tag << 32) | (v + threadIdx.x),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 64) {
      unsigned mn = 0xffffffffu;
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
        mn = 0xffffffffu;
        for (int k = lane; k < n; k += 64) {
          const unsigned long long x =
              __hip_atomic_load(rb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (unsigned)(x >> 32) == tag;
          mn = min(mn, (unsigned)x);
        }
        if (__all(ok)) break;
        if (spins > (1u << 22)) {
          if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return;  // give up (bounded spin): the caller sees the timeout word
        }
        __builtin_amdgcn_s_sleep(1);
      }
      for (int o = 32; o > 0; o >>= 1) mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
      unsigned nv = mn;
      if (dep) {
        // dependent "HBM" load: one line per lane, address from the reduced value
        const size_t idx = ((size_t)(mn + it) * 2654435761ull + (size_t)lane * 8191ull) % nbig;
        const double x = big[idx];
        acc += x;
        nv = mn + (x > 1e300 ? 1u : 0u);
      }
      if (lane == 0) bval = nv;
    }
    __syncthreads();
    v = bval + 1u;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = acc + v;
}

__global__ void trivial(double* out, const double* big, size_t nbig, int dep, int it) {
  if (dep && threadIdx.x < 64) {
    const size_t idx = ((size_t)(it + blockIdx.x) * 2654435761ull + threadIdx.x * 8191ull) % nbig;
    if (big[idx] > 1e300) out[blockIdx.x] = 1.0;
  }
}

int main() {
  const size_t nbig = (size_t)1 << 27;  // 1 GiB of doubles
  double* big;
  CK(hipMalloc(&big, nbig * sizeof(double)));
  CK(hipMemset(big, 0, nbig * sizeof(double)));
  unsigned long long* rec;
  CK(hipMalloc((void**)&rec, 2 * 256 * 16 * sizeof(unsigned long long)));
  unsigned* tmo;
  CK(hipMalloc((void**)&tmo, sizeof(unsigned)));
  double* out;
  CK(hipMalloc(&out, 256 * sizeof(double)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 2000;
  for (int dep = 0; dep < 2; ++dep)
    for (int G : {3, 8})
      for (int B : {32, 64, 128, 256}) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          CK(hipMemsetAsync((void*)rec, 0, 2 * 256 * 16 * sizeof(unsigned long long), s));
          CK(hipMemsetAsync((void*)tmo, 0, sizeof(unsigned), s));
          CK(hipEventRecord(a, s));
          hipLaunchKernelGGL(chain, dim3(B), dim3(256), 0, s, rec, G, (const double*)big, nbig,
                             iters, tmo, out, dep);
          CK(hipGetLastError());
          CK(hipEventRecord(b, s));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          unsigned t = 0;
          CK(hipMemcpy(&t, (void*)tmo, sizeof(unsigned), hipMemcpyDeviceToHost));
          if (t) {
            printf("B=%d G=%d dep=%d: TIMEOUT\n", B, G, dep);
            return 2;
          }
          best = ms < best ? ms : best;
        }
        printf("in-launch exchange: B=%3d G=%d dep_load=%d  %.3f us per exchange\n", B, G, dep,
               1e3 * best / iters);
      }
  // baseline: one launch per phase (kernel boundary + the dependent load)
  for (int dep = 0; dep < 2; ++dep)
    for (int B : {32, 64}) {
      const int n = 2000;
      CK(hipEventRecord(a, s));
      for (int i = 0; i < n; ++i)
        hipLaunchKernelGGL(trivial, dim3(B), dim3(256), 0, s, out, (const double*)big, nbig, dep, i);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("launch per phase:   B=%3d dep_load=%d  %.3f us per launch\n", B, dep, 1e3 * ms / n);
    }
  return 0;
}
