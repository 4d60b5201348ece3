// chain_probe.hip — latency of an in-launch all-to-all exchange (diagnostic).
//
// A persistent grid of B blocks (one per CU) repeats, `iters` times: thread 0
// of every block stores G tagged 8-byte granules {tag, value} (one sc1 store
// each), wave 0 of every block polls all B*G granules (sc1 loads) until every
// tag matches, reduces the values and hands the result to its block through
// LDS.  This is one exchange of the persistent pivot chain (spx_chain.hpp)
// without the phase's work.  Reported: us per exchange, by record layout
// (granule-major planes, or records of 24 B / 64 B / 256 B / 4 KB per block),
// polling passes in flight (1 or 3) and B.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

constexpr int G = 3;
constexpr int MAXB = 256;

// address (in granules) of granule g of block b
__device__ __forceinline__ size_t gaddr(int layout, int g, int b) {
  switch (layout) {
    case 0: return (size_t)g * MAXB + b;   // granule-major planes
    case 1: return (size_t)b * G + g;      // packed 24-B records
    case 2: return (size_t)b * 8 + g;      // 64-B records
    case 3: return (size_t)b * 32 + g;     // 256-B records
    default: return (size_t)b * 512 + g;  // 4-KB records
  }
}

template <int PASSES>
__global__ __launch_bounds__(256) void chain(unsigned long long* rec_, int layout, int iters,
                                             unsigned* tmo_, unsigned* out) {
  gu64* rec = (gu64*)rec_;
  gu32* tmo = (gu32*)tmo_;
  __shared__ unsigned bval;
  __shared__ char pad_lds[96 * 1024];  // one block per CU
  const int lane = threadIdx.x & 63;
  const int B = gridDim.x;
  unsigned v = blockIdx.x;
  if (threadIdx.x == 0) pad_lds[blockIdx.x & 1023] = 0;
  for (int it = 0; it < iters; ++it) {
    const unsigned tag = (unsigned)it + 1u;
    gu64* rb = rec + (size_t)(it & 1) * MAXB * 512;  // two exchanges alternate buffers
    if (threadIdx.x == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g)
        __hip_atomic_store(rb + gaddr(layout, g, blockIdx.x),
                           ((unsigned long long)tag << 32) | (v + g), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 64) {
      const bool live = lane < B;
      const int b = live ? lane : 0;
      unsigned long long x[PASSES][G];
      auto issue = [&](unsigned long long (&g)[G]) {
#pragma unroll
        for (int u = 0; u < G; ++u)
          g[u] = __hip_atomic_load(rb + gaddr(layout, u, b), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
      };
      auto good = [&](const unsigned long long (&g)[G]) {
        bool ok = true;
#pragma unroll
        for (int u = 0; u < G; ++u) ok &= (unsigned)(g[u] >> 32) == tag;
        return __all(ok);
      };
#pragma unroll
      for (int p = 0; p < PASSES; ++p) {
        issue(x[p]);
        if (p + 1 < PASSES) __builtin_amdgcn_s_sleep(8);
      }
      unsigned mn = 0xffffffffu;
      bool done = false;
      for (unsigned spins = 0; !done; ++spins) {
#pragma unroll
        for (int p = 0; p < PASSES; ++p) {
          if (!done) {
            if (good(x[p])) {
              done = true;
              mn = live ? (unsigned)x[p][0] : 0xffffffffu;
            } else {
              issue(x[p]);
            }
          }
        }
        if (!done && spins > (1u << 20)) {
          if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return;  // bounded spin: the caller sees the timeout word
        }
        if (PASSES == 1 && !done) __builtin_amdgcn_s_sleep(1);
      }
      for (int o = 32; o > 0; o >>= 1) mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
      if (lane == 0) bval = mn;
    }
    __syncthreads();
    v = bval + 1u;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = v;
}

int main() {
  unsigned long long* rec;
  const size_t nrec = (size_t)2 * MAXB * 512;
  CK(hipMalloc((void**)&rec, nrec * sizeof(unsigned long long)));
  unsigned* tmo;
  CK(hipMalloc((void**)&tmo, sizeof(unsigned)));
  unsigned* out;
  CK(hipMalloc((void**)&out, MAXB * sizeof(unsigned)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 2000;
  const char* lname[] = {"planes", "rec24B", "rec64B", "rec256B", "rec4KB"};
  for (int passes : {1, 3})
    for (int B : {33, 65})
      for (int layout = 0; layout < 5; ++layout) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          CK(hipMemsetAsync(rec, 0, nrec * sizeof(unsigned long long), s));
          CK(hipMemsetAsync(tmo, 0, sizeof(unsigned), s));
          CK(hipEventRecord(a, s));
          if (passes == 1)
            hipLaunchKernelGGL(chain<1>, dim3(B), dim3(256), 0, s, rec, layout, iters, tmo, out);
          else
            hipLaunchKernelGGL(chain<3>, dim3(B), dim3(256), 0, s, rec, layout, iters, tmo, out);
          CK(hipGetLastError());
          CK(hipEventRecord(b, s));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          unsigned t = 0;
          CK(hipMemcpy(&t, tmo, sizeof(unsigned), hipMemcpyDeviceToHost));
          if (t) {
            printf("B=%d layout=%s passes=%d: TIMEOUT\n", B, lname[layout], passes);
            return 2;
          }
          best = ms < best ? ms : best;
        }
        printf("exchange B=%3d G=%d layout=%-7s passes=%d  %.3f us\n", B, G, lname[layout],
               passes, 1e3 * best / iters);
      }
  return 0;
}
