// xcd_exchange_probe.hip — can the pivot chain run on ONE XCD? (diagnostic)
//
// The persistent pivot chain (spx_chain.hpp) is latency-bound: per pivot two
// all-to-all exchanges among its B blocks and two dependent HBM gathers (a
// column: contiguous; a row: one 8-B load per column, strided by ld).  Its
// blocks are dealt over all 8 XCDs, so every exchange is a cross-XCD round
// trip (write-through sc1 granules).  This probe times one "pivot" of that
// shape:
//     exchange -> column gather -> exchange -> row gather
// for three placements / protocols:
//   spread : B = 64 blocks x 256 threads, dealt over the 8 XCDs, sc1 stores
//   xcd_sc1: 32 blocks x 512 threads on ONE XCD (a 256-block grid, one block
//            per CU by an LDS pin; the blocks read HW_REG_XCC_ID and the first
//            32 on XCD 0 take part, the rest exit), sc1 stores
//   xcd_l2 : the same, plain stores (the granule stays in the XCD's L2, which
//            the consumers' sc1 loads read)
// Every variant polls with sc1 loads, one record of 3 granules per block, one
// pass in flight.  All spins are bounded (a timeout word, the grid drains).
// Output: us per pivot for each (variant, gather) pair, plus a check that every
// participant saw the same exchange results (consistency of the L2 form).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

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
constexpr int64_t M = 8192, NC = 16385, LD = 8448;  // config-3 shape, padded column stride

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// one exchange: every block stores its record (G granules, lane 0 of wave 0),
// wave 0 polls all P records, the block gets min(value) through LDS.
// PLAIN: plain global stores (the line stays in this XCD's L2) instead of sc1.
template <bool PLAIN>
__device__ __forceinline__ bool exchange(gu64* rb, int P, int me, unsigned tag, unsigned v,
                                         unsigned* bval, gu32* tmo) {
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const unsigned long long x = ((unsigned long long)tag << 32) | (v + g);
      if (PLAIN) {
        *((unsigned long long*)(rb + (size_t)g * MAXB + me)) = x;
      } else {
        __hip_atomic_store(rb + (size_t)g * MAXB + me, x, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("" ::: "memory");
  }
  bool ok = true;
  if (threadIdx.x < 64) {
    const bool live = lane < P;
    const int b = live ? lane : 0;
    unsigned mn = 0xffffffffu;
    for (unsigned spins = 0;; ++spins) {
      unsigned long long x[G];
#pragma unroll
      for (int u = 0; u < G; ++u)
        x[u] = __hip_atomic_load(rb + (size_t)u * MAXB + b, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      bool good = true;
#pragma unroll
      for (int u = 0; u < G; ++u) good &= (unsigned)(x[u] >> 32) == tag;
      if (__all(good)) {
        mn = live ? (unsigned)x[0] : 0xffffffffu;
        break;
      }
      if (spins > (1u << 21)) {
        if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        mn = 0xfffffffeu;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    for (int o = 32; o > 0; o >>= 1) mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
    if (lane == 0) *bval = mn;
  }
  __syncthreads();
  return *bval != 0xfffffffeu && ok;
}

// gather: 0 none, 1 column + row (one pivot's two gathers)
template <int CB, bool XCD, bool PLAIN>
__global__ __launch_bounds__(CB) void pivot_probe(unsigned long long* rec_, unsigned* cnt,
                                                  const double* __restrict__ A, int P,
                                                  int gather, int iters, unsigned* tmo_,
                                                  unsigned* out) {
  gu64* rec = (gu64*)rec_;
  gu32* tmo = (gu32*)tmo_;
  __shared__ char pin[96 * 1024];  // one block per CU
  __shared__ int role;
  __shared__ unsigned bval;
  __shared__ unsigned acc[CB / 64];
  const int t = threadIdx.x;
  if (t == 0) pin[blockIdx.x & 1023] = 0;
  int me = blockIdx.x;
  if (XCD) {
    if (t == 0) {
      unsigned x;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
      x &= 7u;
      const unsigned tk = atomicAdd(cnt + x, 1u);
      role = (x == 0u && tk < (unsigned)P) ? (int)tk : -1;
    }
    __syncthreads();
    me = role;
    if (me < 0) return;  // not a participant: this block exits at once
  }
  const int cpb = (int)((NC + P - 1) / P);  // columns per block (one per thread)
  const int rpb = (int)(M / P);             // rows per block
  unsigned v = (unsigned)me;
  for (int it = 0; it < iters; ++it) {
    for (int ph = 0; ph < 2; ++ph) {
      const unsigned tag = 0x80000000u | ((unsigned)it << 1) | (unsigned)ph;
      gu64* rb = rec + (size_t)((2 * it + ph) & 1) * MAXB * 8;
      if (!exchange<PLAIN>(rb, P, me, tag, v, &bval, tmo)) {
        if (t == 0) out[blockIdx.x] = 0xdeadu;
        return;
      }
      unsigned nv = bval + 1u;
      if (gather) {
        const unsigned h = hash32(bval * 2654435761u + (unsigned)(2 * it + ph));
        double x = 0.0;
        if (ph == 0) {  // column gather: rows of this block of column c
          const int64_t c = h % (NC - 1);
          if (t < rpb) x = A[c * LD + (int64_t)me * rpb + t];
        } else {        // row gather: this block's columns of row r
          const int64_t r = h % M;
          const int64_t j = (int64_t)me * cpb + t;
          if (t < cpb && j < NC) x = A[j * LD + r];
        }
        const unsigned any = __ballot(x == 12345.678) != 0ull ? 1u : 0u;
        if ((t & 63) == 0) acc[t >> 6] = any;
        __syncthreads();
        for (int w = 0; w < CB / 64; ++w) nv += acc[w];
      }
      v = nv;
      __syncthreads();
    }
  }
  if (t == 0) out[blockIdx.x] = v;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  unsigned long long* rec;
  CK(hipMalloc((void**)&rec, (size_t)2 * MAXB * 8 * sizeof(unsigned long long)));
  unsigned *cnt, *tmo, *out;
  CK(hipMalloc((void**)&cnt, 8 * sizeof(unsigned)));
  CK(hipMalloc((void**)&tmo, sizeof(unsigned)));
  CK(hipMalloc((void**)&out, MAXB * sizeof(unsigned)));
  double* A;
  const size_t abytes = (size_t)LD * NC * sizeof(double);
  CK(hipMalloc((void**)&A, abytes));
  CK(hipMemset(A, 0, abytes));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct V {
    const char* name;
    int grid, P, cb;
    bool xcd, plain;
  } vars[] = {{"spread_sc1", 64, 64, 256, false, false},
              {"xcd_sc1", 256, 32, 512, true, false},
              {"xcd_l2", 256, 32, 512, true, true},
              {"xcd16_l2", 256, 16, 1024, true, true}};
  for (int gather = 0; gather < 2; ++gather)
    for (const V& x : vars) {
      float best = 1e30f;
      bool fail = false;
      unsigned ref = 0;
      bool consistent = true;
      for (int rep = 0; rep < 3 && !fail; ++rep) {
        CK(hipMemsetAsync(rec, 0, (size_t)2 * MAXB * 8 * sizeof(unsigned long long), s));
        CK(hipMemsetAsync(cnt, 0, 8 * sizeof(unsigned), s));
        CK(hipMemsetAsync(tmo, 0, sizeof(unsigned), s));
        CK(hipMemsetAsync(out, 0xff, MAXB * sizeof(unsigned), s));
        CK(hipEventRecord(a, s));
        if (!x.xcd)
          hipLaunchKernelGGL((pivot_probe<256, false, false>), dim3(x.grid), dim3(256), 0, s, rec,
                             cnt, A, x.P, gather, iters, tmo, out);
        else if (x.cb == 512 && !x.plain)
          hipLaunchKernelGGL((pivot_probe<512, true, false>), dim3(x.grid), dim3(512), 0, s, rec,
                             cnt, A, x.P, gather, iters, tmo, out);
        else if (x.cb == 512)
          hipLaunchKernelGGL((pivot_probe<512, true, true>), dim3(x.grid), dim3(512), 0, s, rec,
                             cnt, A, x.P, gather, iters, tmo, out);
        else
          hipLaunchKernelGGL((pivot_probe<1024, true, true>), dim3(x.grid), dim3(1024), 0, s,
                             rec, cnt, A, x.P, gather, iters, tmo, out);
        CK(hipGetLastError());
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        unsigned tm = 0;
        CK(hipMemcpy(&tm, tmo, sizeof(unsigned), hipMemcpyDeviceToHost));
        unsigned o[MAXB];
        CK(hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost));
        // participants' final values must agree (the exited blocks left 0xffffffff)
        int seen = 0;
        for (int i = 0; i < x.grid; ++i) {
          if (o[i] == 0xffffffffu) continue;
          if (o[i] == 0xdeadu) consistent = false;
          if (!seen++) ref = o[i];
          else if (o[i] != ref) consistent = false;
        }
        if (tm || seen != x.P) {
          printf("%-10s gather=%d: TIMEOUT or missing participants (seen %d of %d)\n", x.name,
                 gather, seen, x.P);
          fail = true;
          break;
        }
        best = ms < best ? ms : best;
      }
      if (!fail)
        printf("%-10s P=%3d CB=%4d gather=%d  %.3f us per pivot (2 exchanges%s)  consistent=%d\n",
               x.name, x.P, x.cb, gather, 1e3 * best / iters, gather ? " + 2 gathers" : "",
               consistent ? 1 : 0);
      fflush(stdout);
    }
  return 0;
}
