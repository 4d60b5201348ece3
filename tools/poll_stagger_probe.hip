// poll_stagger_probe.hip — does a second poll pass in flight shorten the
// chain's exchange? (diagnostic)
//
// The persistent chain's wave 0 polls the B record headers with ONE pass of
// sc1 loads in flight (spx_chain.hpp poll_records_n): a record that lands just
// after a pass read its address waits for the next pass, so detection costs
// up to one load round trip after arrival.  Here the poll keeps TWO passes in
// flight, the second started STAG x 64 cycles (s_sleep) after the first and
// each reissued as soon as it was checked, so a landed record is seen about
// half a round trip sooner -- if the extra loads do not slow the round trip
// itself.  (A first form that slept STAG between the passes inside the loop
// only lengthened it: every stagger slower, profiles/r04/poll_stagger_probe.log;
// this form: profiles/r04/poll_stagger_probe2.log.)  The probe times one
// "pivot" of the chain's shape (exchange -> column gather -> exchange -> row gather, 64
// blocks x 256 threads dealt over the 8 XCDs, 3-granule records, sc1 stores
// and loads) for STAG = 0 (one pass, the chain's poll) and 4 / 8 / 16 / 24.
// Every spin is bounded (a timeout word; the grid drains).
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
constexpr int P = 64;      // blocks
constexpr int MAXB = 256;  // record plane stride
constexpr int64_t M = 8192, NC = 16385, LD = 8448;

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__device__ __forceinline__ void issue(unsigned long long (&x)[G], const gu64* rb, int b) {
#pragma unroll
  for (int u = 0; u < G; ++u)
    x[u] = __hip_atomic_load(rb + (size_t)u * MAXB + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool good(const unsigned long long (&x)[G], unsigned tag) {
  bool g = true;
#pragma unroll
  for (int u = 0; u < G; ++u) g &= (unsigned)(x[u] >> 32) == tag;
  return __all(g);
}

template <int STAG>
__device__ __forceinline__ bool exchange(gu64* rb, int me, unsigned tag, unsigned v,
                                         unsigned* bval, gu32* tmo) {
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g)
      __hip_atomic_store(rb + (size_t)g * MAXB + me, ((unsigned long long)tag << 32) | (v + g),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::: "memory");
  }
  bool ok = true;
  if (threadIdx.x < 64) {
    unsigned long long a[G], c[G];
    unsigned mn = 0xfffffffeu;
    issue(a, rb, lane);
    if (STAG > 0) __builtin_amdgcn_s_sleep(STAG);  // the second pass starts STAG later
    for (unsigned spins = 0;; ++spins) {
      if (STAG > 0) {
        // the passes stay STAG x 64 cycles apart: each is reissued as soon as
        // it has been checked, while the other is in flight (no sleep here)
        issue(c, rb, lane);
        if (good(a, tag)) { mn = (unsigned)a[0]; break; }
        issue(a, rb, lane);
        if (good(c, tag)) { mn = (unsigned)c[0]; break; }
      } else {
        if (good(a, tag)) { mn = (unsigned)a[0]; break; }
        __builtin_amdgcn_s_sleep(1);
        issue(a, rb, lane);
      }
      if (spins > (1u << 20)) {
        if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        mn = 0xfffffffeu;
        break;
      }
    }
    if (ok)
      for (int o = 32; o > 0; o >>= 1) mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
    if (lane == 0) *bval = mn;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no pass left in flight
  }
  __syncthreads();
  return *bval != 0xfffffffeu;
}

template <int STAG>
__global__ __launch_bounds__(256) void pivot_probe(unsigned long long* rec_, const double* A,
                                                   int gather, int iters, unsigned* tmo_,
                                                   unsigned* out) {
  gu64* rec = (gu64*)rec_;
  gu32* tmo = (gu32*)tmo_;
  __shared__ char pin[96 * 1024];  // one block per CU
  __shared__ unsigned bval;
  __shared__ unsigned acc[4];
  const int t = threadIdx.x;
  if (t == 0) pin[blockIdx.x & 1023] = 0;
  const int me = blockIdx.x;
  const int cpb = (int)((NC + P - 1) / P), rpb = (int)(M / P);
  unsigned v = (unsigned)me;
  for (int it = 0; it < iters; ++it) {
    for (int ph = 0; ph < 2; ++ph) {
      const unsigned tag = 0x80000000u | ((unsigned)it << 1) | (unsigned)ph;
      gu64* rb = rec + (size_t)((2 * it + ph) & 1) * MAXB * 8;
      if (!exchange<STAG>(rb, me, tag, v, &bval, tmo)) {
        if (t == 0) out[me] = 0xdeadu;
        return;
      }
      unsigned nv = bval + 1u;
      if (gather) {
        const unsigned h = hash32(bval * 2654435761u + (unsigned)(2 * it + ph));
        double x = 0.0;
        if (ph == 0) {
          const int64_t c = h % (NC - 1);
          if (t < rpb) x = A[c * LD + (int64_t)me * rpb + t];
        } else {
          const int64_t r = h % M;
          const int64_t j = (int64_t)me * cpb + t;
          if (t < cpb && j < NC) x = A[j * LD + r];
        }
        const unsigned any = __ballot(x == 12345.678) != 0ull ? 1u : 0u;
        if ((t & 63) == 0) acc[t >> 6] = any;
        __syncthreads();
        for (int w = 0; w < 4; ++w) nv += acc[w];
      }
      v = nv;
      __syncthreads();
    }
  }
  if (t == 0) out[me] = v;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  unsigned long long* rec;
  CK(hipMalloc((void**)&rec, (size_t)2 * MAXB * 8 * sizeof(unsigned long long)));
  unsigned *tmo, *out;
  CK(hipMalloc((void**)&tmo, sizeof(unsigned)));
  CK(hipMalloc((void**)&out, P * sizeof(unsigned)));
  double* A;
  const size_t abytes = (size_t)LD * NC * sizeof(double);
  CK(hipMalloc((void**)&A, abytes));
  CK(hipMemset(A, 0, abytes));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int stags[] = {0, 4, 8, 16, 24};
  for (int round = 0; round < 2; ++round)
    for (int gather = 0; gather < 2; ++gather)
      for (int st : stags) {
        float best = 1e30f;
        bool fail = false, consistent = true;
        for (int rep = 0; rep < 3 && !fail; ++rep) {
          CK(hipMemsetAsync(rec, 0, (size_t)2 * MAXB * 8 * sizeof(unsigned long long), s));
          CK(hipMemsetAsync(tmo, 0, sizeof(unsigned), s));
          CK(hipEventRecord(a, s));
          switch (st) {
            case 0: hipLaunchKernelGGL(pivot_probe<0>, dim3(P), dim3(256), 0, s, rec, A, gather, iters, tmo, out); break;
            case 4: hipLaunchKernelGGL(pivot_probe<4>, dim3(P), dim3(256), 0, s, rec, A, gather, iters, tmo, out); break;
            case 8: hipLaunchKernelGGL(pivot_probe<8>, dim3(P), dim3(256), 0, s, rec, A, gather, iters, tmo, out); break;
            case 16: hipLaunchKernelGGL(pivot_probe<16>, dim3(P), dim3(256), 0, s, rec, A, gather, iters, tmo, out); break;
            default: hipLaunchKernelGGL(pivot_probe<24>, dim3(P), dim3(256), 0, s, rec, A, gather, iters, tmo, out); break;
          }
          CK(hipGetLastError());
          CK(hipEventRecord(b, s));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          unsigned tm = 0, o[P];
          CK(hipMemcpy(&tm, tmo, sizeof(unsigned), hipMemcpyDeviceToHost));
          CK(hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost));
          for (int i = 1; i < P; ++i) consistent &= o[i] == o[0] && o[i] != 0xdeadu;
          if (tm) {
            printf("stag=%2d gather=%d: TIMEOUT\n", st, gather);
            fail = true;
          }
          best = ms < best ? ms : best;
        }
        if (!fail)
          printf("round %d  stag=%2d gather=%d  %.3f us per pivot (2 exchanges%s)  consistent=%d\n",
                 round, st, gather, 1e3 * best / iters, gather ? " + 2 gathers" : "",
                 consistent ? 1 : 0);
        fflush(stdout);
      }
  return 0;
}
