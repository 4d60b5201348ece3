// two_level_probe.hip — a two-level exchange for the spread chain? (diagnostic)
//
// The spread chain's exchange is an all-to-all among 64 blocks dealt over the
// 8 XCDs: every block stores a 3-granule record write-through (sc1) and every
// block's wave 0 polls all 64 records with sc1 loads -- a cross-XCD round trip
// (spx_chain.hpp poll_records).  VERDICT r3 suggested a two-level form: the 8
// blocks of each XCD first reduce among themselves (records written and read
// on one XCD, as in chain modes 4 / 5), one leader per XCD publishes the XCD's winner
// cross-XCD, and every block polls 8 leader records instead of 64.  This
// probe times both forms on the chain's grid (64 blocks x 256 threads, one
// block per CU by an LDS pin), with and without a dependent gather after each
// exchange, and checks that every block saw the same minimum.  Every spin is
// bounded (a timeout word; the grid drains).
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

constexpr int G = 3;       // granules per record
constexpr int P = 64;      // blocks
constexpr int NX = 8;      // XCDs
constexpr int PL = 256;    // record plane stride
constexpr int64_t M = 8192, NC = 16385, LD = 8448;

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// store one record (G granules) at rb[g * PL + slot], agent scope (the
// chain's stores; the one-XCD modes use the same scope and gain from locality)
__device__ __forceinline__ void put(gu64* rb, int slot, unsigned tag, unsigned v) {
#pragma unroll
  for (int g = 0; g < G; ++g)
    __hip_atomic_store(rb + (size_t)g * PL + slot, ((unsigned long long)tag << 32) | (v + g),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0: poll n records rb[.. + first .. first+n) until every tag matches;
// returns their minimum (0xfffffffe: timed out)
__device__ __forceinline__ unsigned poll_min(const gu64* rb, int first, int n, unsigned tag,
                                             gu32* tmo) {
  const int lane = threadIdx.x & 63;
  const int slot = first + (lane < n ? lane : 0);
  for (unsigned spins = 0;; ++spins) {
    unsigned long long x[G];
#pragma unroll
    for (int u = 0; u < G; ++u)
      x[u] = __hip_atomic_load(rb + (size_t)u * PL + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool good = true;
#pragma unroll
    for (int u = 0; u < G; ++u) good &= (unsigned)(x[u] >> 32) == tag;
    if (__all(good)) {
      unsigned mn = lane < n ? (unsigned)x[0] : 0xffffffffu;
      for (int o = 32; o > 0; o >>= 1) mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
      return mn;
    }
    if (spins > (1u << 21)) {
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return 0xfffffffeu;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

template <bool TWO>
__global__ __launch_bounds__(256) void probe(unsigned long long* rec_, unsigned* cnt,
                                             const double* A, int gather, int iters,
                                             unsigned* tmo_, unsigned* out) {
  gu64* rec = (gu64*)rec_;
  gu32* tmo = (gu32*)tmo_;
  __shared__ char pin[96 * 1024];  // one block per CU
  __shared__ unsigned bval;
  __shared__ int sx, sli;
  __shared__ unsigned acc[4];
  const int t = threadIdx.x;
  if (t == 0) pin[blockIdx.x & 1023] = 0;
  const int me = blockIdx.x;
  if (TWO) {  // my XCD and my index among its blocks
    if (t == 0) {
      unsigned x;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
      x &= 7u;
      sx = (int)x;
      sli = (int)atomicAdd(cnt + x, 1u);
    }
    __syncthreads();
  }
  const int xcd = TWO ? sx : 0, li = TWO ? sli : 0;
  const bool fit = !TWO || li < P / NX;  // (8 blocks per XCD expected; checked on the host)
  const int cpb = (int)((NC + P - 1) / P), rpb = (int)(M / P);
  unsigned v = (unsigned)me;
  for (int it = 0; it < iters && fit; ++it) {
    for (int ph = 0; ph < 2; ++ph) {
      const unsigned tag = 0x80000000u | ((unsigned)it << 1) | (unsigned)ph;
      gu64* half = rec + (size_t)((2 * it + ph) & 1) * PL * 8;
      unsigned mn;
      if (!TWO) {
        if (t == 0) put(half, me, tag, v);
        if (t < 64) mn = poll_min(half, 0, P, tag, tmo);
      } else {
        // level 1: the XCD's 8 records in its L2 (slots xcd*8 + li), then the
        // leader's XCD minimum write-through (slots 128 + xcd)
        if (t == 0) put(half, xcd * 8 + li, tag, v);
        if (t < 64) {
          mn = poll_min(half, xcd * 8, 8, tag, tmo);
          if (li == 0 && (t & 63) == 0 && mn != 0xfffffffeu) put(half, 128 + xcd, tag, mn);
          if (mn != 0xfffffffeu) mn = poll_min(half, 128, NX, tag, tmo);
        }
      }
      if (t == 0) bval = mn;
      __syncthreads();
      if (bval == 0xfffffffeu) {
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
  if (t == 0) out[me] = fit ? v : 0xbeefu;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  unsigned long long* rec;
  CK(hipMalloc((void**)&rec, (size_t)2 * PL * 8 * sizeof(unsigned long long)));
  unsigned *cnt, *tmo, *out;
  CK(hipMalloc((void**)&cnt, NX * sizeof(unsigned)));
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
  for (int round = 0; round < 2; ++round)
    for (int gather = 0; gather < 2; ++gather)
      for (int two = 0; two < 2; ++two) {
        float best = 1e30f;
        bool fail = false, consistent = true;
        for (int rep = 0; rep < 3 && !fail; ++rep) {
          CK(hipMemsetAsync(rec, 0, (size_t)2 * PL * 8 * sizeof(unsigned long long), s));
          CK(hipMemsetAsync(cnt, 0, NX * sizeof(unsigned), s));
          CK(hipMemsetAsync(tmo, 0, sizeof(unsigned), s));
          CK(hipEventRecord(a, s));
          if (two)
            hipLaunchKernelGGL(probe<true>, dim3(P), dim3(256), 0, s, rec, cnt, A, gather, iters, tmo, out);
          else
            hipLaunchKernelGGL(probe<false>, dim3(P), dim3(256), 0, s, rec, cnt, A, gather, iters, tmo, out);
          CK(hipGetLastError());
          CK(hipEventRecord(b, s));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          unsigned tm = 0, o[P], c[NX];
          CK(hipMemcpy(&tm, tmo, sizeof(unsigned), hipMemcpyDeviceToHost));
          CK(hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost));
          CK(hipMemcpy(c, cnt, sizeof(c), hipMemcpyDeviceToHost));
          for (int i = 1; i < P; ++i) consistent &= o[i] == o[0];
          consistent &= o[0] != 0xdeadu && o[0] != 0xbeefu;
          if (two)
            for (int x = 0; x < NX; ++x)
              if (c[x] != P / NX) {
                printf("two-level: XCD %d got %u blocks (8 expected)\n", x, c[x]);
                fail = true;
              }
          if (tm) {
            printf("%s gather=%d: TIMEOUT\n", two ? "two-level" : "one-level", gather);
            fail = true;
          }
          best = ms < best ? ms : best;
        }
        if (!fail)
          printf("round %d  %-9s gather=%d  %.3f us per pivot (2 exchanges%s)  consistent=%d\n",
                 round, two ? "two-level" : "one-level", gather, 1e3 * best / iters,
                 gather ? " + 2 gathers" : "", consistent ? 1 : 0);
        fflush(stdout);
      }
  return 0;
}
