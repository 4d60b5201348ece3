// row_gather_probe.hip — why is the pivot row gather slow from ONE XCD? (diagnostic)
//
// The one-XCD chain (spx_chain.hpp chain_xcd_kernel) cut each exchange from
// ~1.7 to ~0.75 us, but its norm-phase row gather (one 8-B load per column of
// row r of the column-major tableau, 16,385 loads strided by ld) took 2.2-2.8 us
// against 1.1-1.5 us when the chain's blocks are spread over the 8 XCDs
// (profiles/r04/phases_c4.log vs phases_c0.log).  This probe times a loop of
// {exchange -> dependent row gather} for
//   placement: 64 blocks x 256 threads dealt over all XCDs, or 32 x 512 on XCD 0
//   width    : 8 B per column (the current layout), 16 B (column pairs
//              interleaved per row: one load per 2 columns), 32 B (quads)
//   span     : the config-3 stride (ld = 8448 doubles: 1.1 GB), or a compact
//              one (a 64-column-wide stride: the same number of loads in a
//              few MB) -- TLB reach vs DRAM
// and reports us per iteration.  Spins are bounded (timeout word).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
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

constexpr int MAXB = 256;
constexpr int64_t M = 8192, NC = 16385;

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <int CB, bool XCD>
__global__ __launch_bounds__(CB) void row_probe(unsigned long long* rec_, unsigned* cnt,
                                                const double* __restrict__ A, int64_t ld,
                                                int width, int P, int iters, unsigned* tmo_,
                                                unsigned* out) {
  gu64* rec = (gu64*)rec_;
  gu32* tmo = (gu32*)tmo_;
  __shared__ char pin[96 * 1024];
  __shared__ int role;
  __shared__ unsigned bval;
  __shared__ unsigned acc[CB / 64];
  const int t = threadIdx.x, lane = t & 63;
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
    if (me < 0) return;
  }
  // columns per block: NC / (width / 8) "wide columns" of `width` bytes
  const int per = width / 8;
  const int64_t ncw = (NC + per - 1) / per;
  const int64_t cpb = (ncw + P - 1) / P;
  unsigned v = (unsigned)me;
  for (int it = 0; it < iters; ++it) {
    const unsigned tag = 0x80000000u | (unsigned)it;
    gu64* rb = rec + (size_t)(it & 1) * MAXB;
    if (t == 0)
      __hip_atomic_store(rb + me, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED,
                         XCD ? __HIP_MEMORY_SCOPE_WORKGROUP : __HIP_MEMORY_SCOPE_AGENT);
    if (t < 64) {
      unsigned mn = 0xffffffffu;
      for (unsigned spins = 0;; ++spins) {
        const unsigned long long x =
            __hip_atomic_load(rb + (lane < P ? lane : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__all((unsigned)(x >> 32) == tag)) {
          mn = lane < P ? (unsigned)x : 0xffffffffu;
          break;
        }
        if (spins > (1u << 21)) {
          if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          mn = 0xfffffffeu;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      for (int o = 32; o > 0; o >>= 1) mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
      if (lane == 0) bval = mn;
    }
    __syncthreads();
    if (bval == 0xfffffffeu) return;
    const int64_t r = hash32(bval * 2654435761u + (unsigned)it) % M;
    // the row gather: my "wide column" jw's `width` bytes of row r
    const int64_t jw = (int64_t)me * cpb + t;
    bool hit = false;
    if (t < cpb && jw < ncw) {
      // ld < 0: the 512-row panel layout, row r in panel r / 512 of 16 (each
      // panel 512 rows x all columns, a column's piece 4 KiB): span 1.1 GB in
      // all, 67 MB per gather
      const double* p = ld >= 0 ? A + jw * ld * per + r * per
                                : A + (r >> 9) * (512 * ncw * per) + jw * 512 * per + (r & 511) * per;
      if (width == 8) {
        hit = p[0] == 12345.678;
      } else if (width == 16) {
        const double2 x = *reinterpret_cast<const double2*>(p);
        hit = x.x == 12345.678 || x.y == 12345.678;
      } else {
        const double4 x = *reinterpret_cast<const double4*>(p);
        hit = x.x == 12345.678 || x.w == 12345.678;
      }
    }
    const unsigned any = __ballot(hit) != 0ull ? 1u : 0u;
    if (lane == 0) acc[t >> 6] = any;
    __syncthreads();
    unsigned nv = bval + 1u;
    for (int w = 0; w < CB / 64; ++w) nv += acc[w];
    v = nv;
    __syncthreads();
  }
  if (t == 0) out[blockIdx.x] = v;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  unsigned long long* rec;
  CK(hipMalloc((void**)&rec, (size_t)2 * MAXB * sizeof(unsigned long long)));
  unsigned *cnt, *tmo, *out;
  CK(hipMalloc((void**)&cnt, 8 * sizeof(unsigned)));
  CK(hipMalloc((void**)&tmo, sizeof(unsigned)));
  CK(hipMalloc((void**)&out, MAXB * sizeof(unsigned)));
  const int64_t LDF = 8448;  // config 3's padded column stride (doubles)
  // every span's largest address: (wide column ncw-1) * ld * per + (M-1) * per
  // < (NC + 8) * LDF + 2 * M doubles
  const size_t abytes = ((size_t)LDF * (NC + 8) + 2 * (size_t)M + 4096) * sizeof(double);
  double* Ad;  // default hipMalloc
  CK(hipMalloc((void**)&Ad, abytes));
  CK(hipMemset(Ad, 0, abytes));
  double* Ac = nullptr;  // physically contiguous (hipDeviceMallocContiguous): bigger TLB fragments?
  if (hipExtMallocWithFlags((void**)&Ac, abytes, hipDeviceMallocContiguous) != hipSuccess) {
    (void)hipGetLastError();
    Ac = nullptr;
    printf("hipDeviceMallocContiguous: allocation refused\n");
  } else {
    CK(hipMemset(Ac, 0, abytes));
  }
  {
    const int64_t ncw1 = NC, ncw2 = (NC + 1) / 2;
    const int64_t mx1 = (15 * 512 * ncw1 + (ncw1 - 1) * 512 + 511) + 1;
    const int64_t mx2 = (15 * 512 * ncw2 + (ncw2 - 1) * 512 + 511) * 2 + 2;
    if ((size_t)std::max(mx1, mx2) * sizeof(double) > abytes) {
      printf("panels16 exceeds the buffer\n");
      return 2;
    }
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // spans: "1.1GB" the config-3 column stride; "panel" a 512-row panel layout
  // (4 KiB per column: one row gather touches 67 MB); "compact" ~1 MB
  struct Sp { const char* name; int64_t ld8; bool contig; } spans[] = {
      {"1.1GB", LDF, false}, {"1.1GB-contig", LDF, true}, {"panel", 512, false},
      {"panels16", -1, false}, {"compact", 8, false}};
  for (int xcd = 0; xcd < 2; ++xcd)
    for (int width : {8, 16})
      for (const Sp& sp : spans) {
        if (sp.contig && !Ac) continue;
        const double* A = sp.contig ? Ac : Ad;
        const int per = width / 8;
        const int64_t ldd = sp.ld8 == 8 ? (8 / per > 0 ? 8 / per : 1) : sp.ld8;
        // panels16 bound: (15 * 512 * ncw + (ncw - 1) * 512 + 511) * per + per - 1 doubles
        // < 16 * 512 * 16393 * 2 < abytes / 8 (checked on the host below)
        const int P = xcd ? 32 : 64;
        float best = 1e30f;
        bool fail = false;
        for (int rep = 0; rep < 3 && !fail; ++rep) {
          CK(hipMemsetAsync(rec, 0, (size_t)2 * MAXB * sizeof(unsigned long long), s));
          CK(hipMemsetAsync(cnt, 0, 8 * sizeof(unsigned), s));
          CK(hipMemsetAsync(tmo, 0, sizeof(unsigned), s));
          CK(hipEventRecord(a, s));
          if (xcd)
            hipLaunchKernelGGL((row_probe<512, true>), dim3(256), dim3(512), 0, s, rec, cnt, A,
                               ldd, width, P, iters, tmo, out);
          else
            hipLaunchKernelGGL((row_probe<256, false>), dim3(64), dim3(256), 0, s, rec, cnt, A,
                               ldd, width, P, iters, tmo, out);
          CK(hipGetLastError());
          CK(hipEventRecord(b, s));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          unsigned tm = 0;
          CK(hipMemcpy(&tm, tmo, sizeof(unsigned), hipMemcpyDeviceToHost));
          if (tm) {
            printf("%s width=%d span=%s: TIMEOUT\n", xcd ? "xcd32x512" : "spread64x256", width,
                   sp.name);
            fail = true;
          }
          best = ms < best ? ms : best;
        }
        if (!fail)
          printf("%-13s width=%2d B span=%-12s  %.3f us per {exchange + row gather}\n",
                 xcd ? "xcd32x512" : "spread64x256", width, sp.name, 1e3 * best / iters);
        fflush(stdout);
      }
  return 0;
}
