// spx_kernels.hpp — gfx950 (CDNA4) kernels of the dense simplex pivot engine.
//
// One pivot of the tableau method (the loop inside simple_simplex's
// optimize_json_format, called at reference app/controllers/solver_controller.py:318)
// is TWO launches on one stream in steady state:
//
//   norm_kernel  : leaving row r from the ratio partials; pivot row
//                  p = T[r,:] / T[r,c]; objective-row update; compaction of the
//                  columns with p[j] != 0; per-block entering partials for the
//                  NEXT pivot; basis / history bookkeeping.
//   elim_kernel  : T[i,j] <- T[i,j] - F[i]*p[j] over the compacted columns,
//                  row r <- p, column c <- e_r (the HBM-roofline kernel), and,
//                  fused in, the NEXT pivot's ratio test: every block reduces
//                  the entering partials to c'; column group 0 updates columns
//                  c' and RHS of its row chunk itself, snapshots F' = T[:,c']
//                  and writes that chunk's min-ratio partial.
//
// prime_kernel runs once per host call (after a load / objective change /
// forced pivot) to produce the first c, F and ratio partials.
//
// A row-sharded rank (one process per GPU) runs prep_kernel -> ONE all-gather
// -> norm_kernel<FINISH> -> elim_kernel per pivot: prep packs this rank's
// best leaving-row candidate and its normalised row [key | p[0..N)]; after
// the all-gather every rank takes the lexicographic winner's row as p.
//
// Memory layout: the m constraint rows are stored COLUMN-MAJOR
// (column j is ld contiguous doubles), so the ratio test reads two contiguous
// columns, the elimination streams whole columns with 16-B lane accesses, and
// a column whose pivot-row entry is zero is skipped without touching HBM.  The
// objective row lives in its own contiguous vector `obj`.
//
// Arithmetic is fixed to match the oracle bit for bit: IEEE division for p
// and the ratios, separate multiply and subtract (never contracted to FMA),
// lexicographic (value, tie) argmin reductions held in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spx {

constexpr int BLK = 256;  // threads per workgroup (4 wave64)
constexpr int NWAVE = BLK / 64;

// The load's zeroing of a context's small buffers in one launch (spx_load /
// spx_load_rows, alloc_common): span y of the list is cleared by the blocks
// of grid row y, 16-B stores over its 16-B-aligned body (every span starts at
// a hipMalloc'd, 256-B-aligned address) and 4-B stores over the rest.  Replaces
// ~25 fill launches per load (round 6: a textbook LP's load was mostly those).
constexpr int ZERO_SPANS_MAX = 32;
struct ZeroSpans {
  uint32_t* p[ZERO_SPANS_MAX];
  uint64_t words[ZERO_SPANS_MAX];  // 4-B words per span
  int n;
};
__global__ __launch_bounds__(256) void zero_spans_kernel(ZeroSpans z) {
  const int s = blockIdx.y;
  if (s >= z.n) return;
  uint32_t* p = z.p[s];
  const uint64_t w = z.words[s], w4 = w / 4;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  uint4* q = reinterpret_cast<uint4*>(p);
  for (uint64_t i = t0; i < w4; i += step) q[i] = make_uint4(0u, 0u, 0u, 0u);
  for (uint64_t i = w4 * 4 + t0; i < w; i += step) p[i] = 0u;
}

// Row-major <-> column-major transposes of the boundary (spx_load_rows /
// spx_get_tableau with SPX_ROW_MAJOR): 32 x 32 tiles through LDS (a padded
// row, so the column reads do not share a bank), 32 x 8 threads, so both the
// row-major and the column-major side move 256-B runs.  rm: R x C row-major,
// pitch prm doubles; cm: column-major, pitch pcm doubles (element (i, j) at
// cm[j * pcm + i]).  TO_CM: rm -> cm, else cm -> rm.
template <bool TO_CM>
__global__ __launch_bounds__(256) void transpose_kernel(const double* __restrict__ src,
                                                        double* __restrict__ dst, int64_t R,
                                                        int64_t C, int64_t prm, int64_t pcm) {
  __shared__ double tile[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t i0 = (int64_t)blockIdx.y * 32, j0 = (int64_t)blockIdx.x * 32;
  if constexpr (TO_CM) {
    for (int y = ty; y < 32; y += 8) {  // rows i0 + y, columns j0 + tx
      const int64_t i = i0 + y, j = j0 + tx;
      if (i < R && j < C) tile[y][tx] = src[i * prm + j];
    }
    __syncthreads();
    for (int y = ty; y < 32; y += 8) {  // columns j0 + y, rows i0 + tx
      const int64_t i = i0 + tx, j = j0 + y;
      if (i < R && j < C) dst[j * pcm + i] = tile[tx][y];
    }
  } else {
    for (int y = ty; y < 32; y += 8) {  // columns j0 + y, rows i0 + tx
      const int64_t i = i0 + tx, j = j0 + y;
      if (i < R && j < C) tile[tx][y] = src[j * pcm + i];
    }
    __syncthreads();
    for (int y = ty; y < 32; y += 8) {  // rows i0 + y, columns j0 + tx
      const int64_t i = i0 + y, j = j0 + tx;
      if (i < R && j < C) dst[i * prm + j] = tile[y][tx];
    }
  }
}

// device-side solve status (mapped to SPX_* codes on the host)
constexpr int32_t ST_RUNNING = 0;
constexpr int32_t ST_OPTIMAL = 1;
constexpr int32_t ST_UNBOUNDED = 2;
constexpr int32_t ST_LIMIT = 3;

constexpr int32_t RULE_DANTZIG = 0;
constexpr int32_t RULE_BLAND = 1;

struct Params {
  int32_t rule;
  int32_t skip_zero;
  double eps_opt;
  double eps_piv;
  int64_t n_enter;
  int64_t iter_limit;  // absolute pivot count at which norm_kernel stops
};

// Written by exactly one thread of one kernel per pivot, read by the next
// kernels on the stream; no field is written while another block of the same
// launch may still read it.
struct State {
  int32_t status;
  int32_t n_ratio_part;   // valid ratio partials for the pending pivot
  int32_t count[2];       // compacted-column counters, by pivot parity
  int32_t cur;            // parity slot of the pivot being eliminated
  int32_t pad;
  int64_t iters;          // pivots completed since load (elim increments)
  int64_t c;              // entering column of the pivot being eliminated
  int64_t r;              // its leaving row (global index)
  double zc;              // objective-row entry of column c before the pivot
  double piv;             // pivot element (owner rank only)
  int64_t c_next;         // pending entering column (-1: optimal)
  double zc_next;
  int64_t forced_c;       // >= 0: spx_pivot_at column (prime_kernel)
  int64_t forced_r;       // >= 0: spx_pivot_at row (norm_kernel)
  int64_t touched_total;  // sum of compacted columns over pivots (bytes)
  int64_t hist_cap;
  int64_t hs_ticks;       // persistent chains: start-handshake bound (s_memrealtime
                          // ticks, 100 MHz; < 0 forces ABORT, a test hook)
};

// Argmin key in memory (partials).  Smallest v, then smallest t; `row`
// carries the payload.  t is unique among candidates, so every reduction
// order gives the same answer.
struct Key {
  double v;
  int64_t t;
  int64_t row;
  int64_t pad;
};

// The same key in registers: component-wise selects only (a select of the
// whole struct made hipcc spill it to scratch).
struct KeyR {
  double v;
  int64_t t;
  int64_t row;
};

__device__ __forceinline__ KeyR keyr_none() { return KeyR{__builtin_inf(), INT64_MAX, -1}; }

__device__ __forceinline__ void kmin(KeyR& a, double v, int64_t t, int64_t row) {
  const bool take = (v < a.v) || (v == a.v && t < a.t);
  a.v = take ? v : a.v;
  a.t = take ? t : a.t;
  a.row = take ? row : a.row;
}

__device__ __forceinline__ void wave_min(KeyR& k) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double v = __shfl_xor(k.v, off, 64);
    const int64_t t = __shfl_xor(k.t, off, 64);
    const int64_t row = __shfl_xor(k.row, off, 64);
    kmin(k, v, t, row);
  }
}

// The same wave argmin without LDS: DPP row rotations / quad permutes inside
// each row of 16 lanes, then the gfx950 permlane swaps for lanes 16 and 32
// apart.  Every lane receives the result.  (__shfl_xor is a ds_bpermute per
// dword: six dependent LDS round trips, ~0.7 us on the lazy kernels' path.)
template <int CTRL>
__device__ __forceinline__ int64_t dpp64(int64_t x) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(x & 0xffffffff), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(x >> 32), CTRL, 0xf, 0xf, false);
  return ((int64_t)hi << 32) | (uint32_t)lo;
}
template <int CTRL>
__device__ __forceinline__ void kmin_dpp(KeyR& k) {
  const double v = __longlong_as_double(dpp64<CTRL>(__double_as_longlong(k.v)));
  const int64_t t = dpp64<CTRL>(k.t);
  const int64_t row = dpp64<CTRL>(k.row);
  kmin(k, v, t, row);
}
// partner value `d` lanes away (d = 16 or 32) from the permlane swap pair
template <int D>
__device__ __forceinline__ int64_t swap64(int64_t x) {
  const unsigned lo = (unsigned)(x & 0xffffffff), hi = (unsigned)(x >> 32);
  const bool upper = (threadIdx.x & D) != 0;
  unsigned plo, phi;
  if constexpr (D == 16) {
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    plo = upper ? a[0] : a[1];
    phi = upper ? b[0] : b[1];
  } else {
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    plo = upper ? a[0] : a[1];
    phi = upper ? b[0] : b[1];
  }
  return ((int64_t)phi << 32) | plo;
}
template <int D>
__device__ __forceinline__ void kmin_swap(KeyR& k) {
  const double v = __longlong_as_double(swap64<D>(__double_as_longlong(k.v)));
  const int64_t t = swap64<D>(k.t);
  const int64_t row = swap64<D>(k.row);
  kmin(k, v, t, row);
}
__device__ __forceinline__ void wave_min_dpp(KeyR& k) {
  kmin_dpp<0x128>(k);  // row_ror:8
  kmin_dpp<0x124>(k);  // row_ror:4
  kmin_dpp<0x4E>(k);   // quad_perm [2,3,0,1]
  kmin_dpp<0xB1>(k);   // quad_perm [1,0,3,2]
  kmin_swap<16>(k);
  kmin_swap<32>(k);
}

// Block-wide argmin; every thread receives the result.
__device__ __forceinline__ KeyR block_min(KeyR k) {
  __shared__ double sv[NWAVE];
  __shared__ int64_t st_[NWAVE];
  __shared__ int64_t sr[NWAVE];
  wave_min(k);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = k.v;
    st_[w] = k.t;
    sr[w] = k.row;
  }
  __syncthreads();
  KeyR r{sv[0], st_[0], sr[0]};
#pragma unroll
  for (int i = 1; i < NWAVE; ++i) kmin(r, sv[i], st_[i], sr[i]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ KeyR reduce_keys(const Key* __restrict__ part, int n) {
  KeyR k = keyr_none();
  for (int i = threadIdx.x; i < n; i += BLK) kmin(k, part[i].v, part[i].t, part[i].row);
  return block_min(k);
}

__device__ __forceinline__ void store_key(Key* dst, const KeyR& k) {
  Key o;
  o.v = k.v;
  o.t = k.t;
  o.row = k.row;
  o.pad = 0;
  *dst = o;
}

// Round-to-nearest multiply then subtract: never contracted to FMA.
__device__ __forceinline__ double msub(double t, double f, double p) {
  return __dsub_rn(t, __dmul_rn(f, p));
}

// One candidate row of the min-ratio test.
__device__ __forceinline__ void ratio_candidate(KeyR& k, double fv, double bv, int64_t grow,
                                                const int64_t* __restrict__ basis, int32_t rule,
                                                double eps_piv) {
  if (fv > eps_piv) {
    const double q = bv / fv;
    if (q == q) kmin(k, q, (rule == RULE_BLAND) ? basis[grow] : grow, grow);
  }
}

typedef double dbl2 __attribute__((ext_vector_type(2)));

// v_readlane of a double held per lane (lane index wave-uniform).
__device__ __forceinline__ double rdlane(double v, int lane) {
  const int64_t b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}

template <bool NT>
__device__ __forceinline__ dbl2 ld2(const double* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(p));
  return *reinterpret_cast<const dbl2*>(p);
}
template <bool NT>
__device__ __forceinline__ void st2(double* p, dbl2 v) {
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(p));
  else *reinterpret_cast<dbl2*>(p) = v;
}

// ---------------------------------------------------------------------------
// prime_kernel: pending entering column c (rule, or forced) + snapshot
// F[slot] = T[:,c] + min-ratio partials.  grid: NBr blocks, grid-stride.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(BLK) void prime_kernel(const double* __restrict__ A, int64_t ld,
                                                    int64_t m_local, int64_t row0, int64_t N,
                                                    const double* __restrict__ obj,
                                                    double* __restrict__ F2,
                                                    const Key* __restrict__ enter_part, int nbn,
                                                    Key* __restrict__ ratio_part,
                                                    const int64_t* __restrict__ basis,
                                                    const Params* __restrict__ prm, State* st) {
  if (st->status != ST_RUNNING) return;
  const int32_t rule = prm->rule;
  const double eps_piv = prm->eps_piv;
  const int64_t forced_c = st->forced_c;
  const int slot = (int)(st->iters & 1);
  int64_t c;
  if (forced_c >= 0) {
    c = forced_c;
  } else {
    const KeyR e = reduce_keys(enter_part, nbn);
    if (e.row < 0) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->status = ST_OPTIMAL;
        st->c_next = -1;
      }
      return;
    }
    c = e.row;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->c_next = c;
    st->zc_next = obj[c];
    st->count[slot] = 0;
    st->n_ratio_part = gridDim.x;
  }
  double* __restrict__ F = F2 + slot * ld;
  const double* __restrict__ colc = A + c * ld;
  const double* __restrict__ rhs = A + (N - 1) * ld;
  KeyR k = keyr_none();
  const bool forced = forced_c >= 0;
  for (int64_t i = ((int64_t)blockIdx.x * BLK + threadIdx.x) * 2; i < m_local;
       i += (int64_t)gridDim.x * BLK * 2) {
    const dbl2 fv = ld2<false>(colc + i);
    const dbl2 bv = ld2<false>(rhs + i);
    st2<false>(F + i, fv);
    if (!forced) {
      ratio_candidate(k, fv.x, bv.x, row0 + i, basis, rule, eps_piv);
      if (i + 1 < m_local) ratio_candidate(k, fv.y, bv.y, row0 + i + 1, basis, rule, eps_piv);
    }
  }
  k = block_min(k);
  if (threadIdx.x == 0) store_key(ratio_part + blockIdx.x, k);
}

// ---------------------------------------------------------------------------
// norm_kernel: one thread per tableau column.
//   MODE_FUSED  (1 rank): leaving row from ratio partials, p, objective,
//                         compaction, entering partials, bookkeeping.
//   MODE_FINISH (sharded, after the all-gather): leaving row = the winner of
//                         the gathered per-rank keys, p = the winner's row;
//                         then as FUSED.
//   MODE_INIT   entering partials only (start of every host call).
// ---------------------------------------------------------------------------
constexpr int MODE_FUSED = 0;
constexpr int MODE_FINISH = 2;
constexpr int MODE_INIT = 3;

// Layout of one rank's all-gather payload: a Key, then p[0..N).
constexpr int64_t PAYLOAD_HDR = 32;

template <int MODE>
__global__ __launch_bounds__(BLK) void norm_kernel(const double* __restrict__ A, int64_t ld,
                                                   int64_t m_local, int64_t row0, int64_t N,
                                                   double* __restrict__ obj,
                                                   const double* __restrict__ F2,
                                                   double* __restrict__ P, int* __restrict__ list,
                                                   const Key* __restrict__ keys,
                                                   const char* __restrict__ gbuf,
                                                   int64_t gstride, int nranks,
                                                   Key* __restrict__ enter_part,
                                                   int64_t* __restrict__ basis,
                                                   int64_t* __restrict__ hist,
                                                   const Params* __restrict__ prm, State* st) {
  if (MODE != MODE_INIT && st->status != ST_RUNNING) return;
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  const int32_t rule = prm->rule;
  const double eps_opt = prm->eps_opt;
  const int64_t n_enter = prm->n_enter;
  const bool skip = prm->skip_zero != 0;
  const int64_t it = st->iters;
  const int slot = (int)(it & 1);
  const int64_t c = (MODE == MODE_INIT) ? -1 : st->c_next;
  const int64_t forced_r = st->forced_r;
  // independent of the leaving row: in flight during the ratio reduction
  double o = (j < N) ? obj[j] : 0.0;

  int64_t r = -1;
  const double* __restrict__ pw = nullptr;  // FINISH: the winner's p row
  if (MODE == MODE_FUSED || MODE == MODE_FINISH) {
    // FINISH: a time-limit stop requested by rank 0's host rides in rank 0's
    // payload header, so every rank stops before the same pivot
    const bool stop_req =
        MODE == MODE_FINISH && (reinterpret_cast<const Key*>(gbuf)->pad >> 32) != 0;
    if (c < 0 || (forced_r < 0 && (it >= prm->iter_limit || stop_req))) {
      if (blockIdx.x == 0 && threadIdx.x == 0) st->status = (c < 0) ? ST_OPTIMAL : ST_LIMIT;
      return;
    }
    if (MODE == MODE_FUSED) {
      r = forced_r;
      if (r < 0) {
        const KeyR rk = reduce_keys(keys, st->n_ratio_part);
        if (rk.row < 0) {
          if (blockIdx.x == 0 && threadIdx.x == 0) st->status = ST_UNBOUNDED;
          return;
        }
        r = rk.row;
      }
    } else {
      // lexicographic winner over the ranks' keys (t is unique, so exactly
      // one rank's key equals the minimum; its payload holds p)
      KeyR rk = keyr_none();
      for (int q = threadIdx.x; q < nranks; q += BLK) {
        const Key* kq = reinterpret_cast<const Key*>(gbuf + q * gstride);
        kmin(rk, kq->v, kq->t, kq->row);
      }
      rk = block_min(rk);
      if (rk.row < 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) st->status = ST_UNBOUNDED;
        return;
      }
      r = rk.row;
      int w = 0;
      for (int q = 0; q < nranks; ++q) {
        const Key* kq = reinterpret_cast<const Key*>(gbuf + q * gstride);
        if (kq->row == r && kq->v == rk.v && kq->t == rk.t) {
          w = q;
          break;
        }
      }
      pw = reinterpret_cast<const double*>(gbuf + w * gstride + PAYLOAD_HDR);
    }
  }
  const double* __restrict__ F = F2 + slot * ld;

  bool nz = false;
  KeyR ek = keyr_none();
  const double zc = st->zc_next;
  if (j < N) {
    if (MODE != MODE_INIT) {
      double p;
      if (MODE == MODE_FUSED) p = A[j * ld + (r - row0)] / F[r - row0];
      else p = pw[j];
      P[j] = p;
      nz = (p != 0.0) || !skip;
      if (j == c) {
        o = 0.0;
      } else if (nz) {
        o = msub(o, zc, p);
      }
      obj[j] = o;
    }
    if (j < n_enter && o < -eps_opt) kmin(ek, (rule == RULE_BLAND) ? 0.0 : o, j, j);
  }

  if (MODE != MODE_INIT) {
    // stream compaction of the columns the elimination must touch
    __shared__ int wcount[NWAVE];
    __shared__ int wbase[NWAVE];
    __shared__ int bbase;
    const unsigned long long mask = __ballot(nz);
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int wpre = __popcll(mask & ((1ull << lane) - 1ull));
    if (lane == 0) wcount[w] = __popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
      int s = 0;
#pragma unroll
      for (int q = 0; q < NWAVE; ++q) {
        wbase[q] = s;
        s += wcount[q];
      }
      bbase = s ? atomicAdd(&st->count[slot], s) : 0;
    }
    __syncthreads();
    if (nz) list[bbase + wbase[w] + wpre] = (int)j;
  }

  ek = block_min(ek);
  if (threadIdx.x == 0) store_key(enter_part + blockIdx.x, ek);

  if (MODE != MODE_INIT && blockIdx.x == 0 && threadIdx.x == 0) {
    st->r = r;
    if (r - row0 >= 0 && r - row0 < m_local) st->piv = F[r - row0];
    st->c = c;
    st->zc = zc;
    st->cur = slot;
    basis[r] = c;
    if (it < st->hist_cap) {
      hist[2 * it] = r;
      hist[2 * it + 1] = c;
    }
  }
}

// Time-limit stop of a sharded solve (spx_solve): rank 0's host sets a word of
// pinned host memory; rank 0's payload header carries it (Key.pad bit 32) to
// every rank, which stop before the same pivot (status ST_LIMIT).
__device__ __forceinline__ bool stop_requested(int rank, const int32_t* stop_req) {
  return rank == 0 && stop_req &&
         __hip_atomic_load(const_cast<int32_t*>(stop_req), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

// prep_kernel (sharded rank): this rank's leaving-row candidate for the
// pending pivot and its normalised row, packed as the all-gather payload
// [Key (pad = rank) | p[0..N)].  One thread per column.  A forced pivot
// (spx_pivot_at) is published by the rank that owns the forced row.
__global__ __launch_bounds__(BLK) void prep_kernel(const double* __restrict__ A, int64_t ld,
                                                   int64_t m_local, int64_t row0, int64_t N,
                                                   const double* __restrict__ F2,
                                                   const Key* __restrict__ ratio_part,
                                                   char* __restrict__ sendbuf, int rank,
                                                   const State* st,
                                                   const int32_t* stop_req) {
  const bool live = st->status == ST_RUNNING && st->c_next >= 0;
  const int64_t forced_r = st->forced_r;
  KeyR k = keyr_none();
  if (forced_r >= 0) {
    if (forced_r >= row0 && forced_r < row0 + m_local) k = KeyR{0.0, 0, forced_r};
  } else {
    k = reduce_keys(ratio_part, live ? st->n_ratio_part : 0);
  }
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  const double* __restrict__ F = F2 + (st->iters & 1) * ld;
  double* __restrict__ p = reinterpret_cast<double*>(sendbuf + PAYLOAD_HDR);
  if (live && k.row >= 0 && j < N) {
    const int64_t rl = k.row - row0;
    p[j] = A[j * ld + rl] / F[rl];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    Key o;
    o.v = k.v;
    o.t = k.t;
    o.row = live ? k.row : -1;
    o.pad = rank | ((int64_t)stop_requested(rank, stop_req) << 32);
    if (!live) {
      o.v = __builtin_inf();
      o.t = INT64_MAX;
    }
    *reinterpret_cast<Key*>(sendbuf) = o;
  }
}

// ---------------------------------------------------------------------------
// elim_kernel: the rank-1 Gauss-Jordan update (HBM-bound) + the next pivot's
// ratio test.  grid = rch * G blocks; block b owns row chunk (b % rch) of
// RC = BLK*R rows and column group g = b / rch.  Each thread keeps its R values
// of F in registers and streams R/2 16-B vectors per column, two columns in
// flight.  Groups 1..G-1 (all groups if G == 1) share the compacted column
// list, either in contiguous ranges or interleaved (ILV: at any moment the
// active blocks sweep a contiguous window of the list).  Group 0 updates the
// pending entering column c' and the RHS of its chunk, snapshots F' and writes
// the chunk's ratio partial for the next pivot.  NTL / NTS select
// non-temporal loads / stores for the once-touched stream.
// ---------------------------------------------------------------------------
template <int R, bool NTL, bool NTS>
struct Elim {
  static constexpr int V = R / 2;

  __device__ static void load(const double* __restrict__ col, dbl2 (&t)[V],
                              const bool (&ok)[V], int64_t base) {
#pragma unroll
    for (int v = 0; v < V; ++v)
      if (ok[v]) t[v] = ld2<NTL>(col + base + (int64_t)v * BLK * 2);
  }

  __device__ static void update(double* __restrict__ col, const dbl2 (&t)[V],
                                const dbl2 (&f)[V], const bool (&ok)[V], int64_t base,
                                int64_t rl, double pj, dbl2 (&out)[V]) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int64_t i = base + (int64_t)v * BLK * 2;
      if (ok[v]) {
        dbl2 o;
        o.x = (i == rl) ? pj : msub(t[v].x, f[v].x, pj);
        o.y = (i + 1 == rl) ? pj : msub(t[v].y, f[v].y, pj);
        out[v] = o;
        st2<NTS>(col + i, o);
      }
    }
  }

  __device__ static void unit(double* __restrict__ col, const bool (&ok)[V], int64_t base,
                              int64_t rl) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int64_t i = base + (int64_t)v * BLK * 2;
      if (ok[v]) {
        dbl2 o;
        o.x = (i == rl) ? 1.0 : 0.0;
        o.y = (i + 1 == rl) ? 1.0 : 0.0;
        st2<NTS>(col + i, o);
      }
    }
  }
};

// Walks one column group's share of the compacted list: 64 entries at a time
// held in lanes (one vector load of list[] + one gather of P[] per window),
// read with v_readlane so the stream loop issues no dependent scalar loads.
// Columns c' and RHS are skipped (group 0 owns them).  Wave-uniform.
struct ListCursor {
  const int* __restrict__ list;
  const double* __restrict__ P;
  int w0, ke, step, q, nwin, jl;
  double pl;
  int64_t cn, rhs;

  __device__ void load_window(int lane) {
    const int kk = w0 + lane * step;
    jl = -1;
    pl = 0.0;
    if (kk < ke) {
      jl = list[kk];
      pl = P[jl];
    }
    nwin = w0 < ke ? min(64, (ke - w0 + step - 1) / step) : 0;
    q = 0;
  }

  __device__ bool next(int& j, double& p, int lane) {
    for (;;) {
      for (; q < nwin; ++q) {
        const int jj = __builtin_amdgcn_readlane(jl, q);
        if (jj != cn && jj != rhs) {
          j = jj;
          p = rdlane(pl, q);
          ++q;
          return true;
        }
      }
      if (nwin == 0) return false;
      w0 += 64 * step;
      if (w0 >= ke) {
        nwin = 0;
        return false;
      }
      load_window(lane);
    }
  }
};

template <int R, bool NTL, bool NTS, bool ILV, bool PIPE>
__global__ __launch_bounds__(BLK) void elim_kernel(
    double* __restrict__ A, int64_t ld, int64_t m_local, int64_t row0, int64_t N,
    double* __restrict__ F2, const double* __restrict__ P, const int* __restrict__ list, int rch,
    int G, const Key* __restrict__ enter_part, int nbn, Key* __restrict__ ratio_part,
    const double* __restrict__ obj, const int64_t* __restrict__ basis,
    const Params* __restrict__ prm, State* st, int xcd_swz) {
  static_assert(R % 2 == 0, "R must be even");
  using E = Elim<R, NTL, NTS>;
  constexpr int V = R / 2;
  if (st->status != ST_RUNNING) return;
  const int cur = st->cur;
  const int count = st->count[cur];
  const int64_t c = st->c;
  const int64_t rl = st->r - row0;
  const int64_t rhs = N - 1;
  const bool skip = prm->skip_zero != 0;
  // xcd_swz: blocks are dealt round-robin over the 8 XCDs, so remap physical
  // block b to logical (b % 8) * (grid / 8) + b / 8: each XCD then streams
  // whole columns (all row chunks) instead of one chunk of every column
  int bid = blockIdx.x;
  if (xcd_swz && (gridDim.x & 7) == 0) bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const int chunk = bid % rch;
  const int g = bid / rch;
  const double* __restrict__ F = F2 + cur * ld;

  // Issue the loads that do not depend on c' first (pivot-column values of
  // this chunk, the first 64-entry window of this group's column list and the
  // matching p values), so they are in flight during the c' reduction.
  const int64_t base = (int64_t)chunk * BLK * R + threadIdx.x * 2;
  dbl2 f[V];
  bool ok[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int64_t i = base + (int64_t)v * BLK * 2;
    ok[v] = i < m_local;
    f[v] = ok[v] ? ld2<false>(F + i) : dbl2{0.0, 0.0};
  }
  const int LG = G > 1 ? G - 1 : 1;
  const int lg = G > 1 ? g - 1 : 0;
  int kb = 0, ke = 0, step = 1;
  if (lg >= 0) {
    if (ILV) {
      kb = lg;
      ke = count;
      step = LG;
    } else {
      kb = (int)(((int64_t)lg * count) / LG);
      ke = (int)(((int64_t)(lg + 1) * count) / LG);
    }
  }
  const int lane = threadIdx.x & 63;
  ListCursor cur_l{list, P, kb, ke, step, 0, 0, -1, 0.0, -1, rhs};
  if (lg >= 0) cur_l.load_window(lane);

  // the next pivot's entering column: every block must leave it (and the RHS)
  // to group 0
  const int64_t cn = reduce_keys(enter_part, nbn).row;
  cur_l.cn = cn;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->iters += 1;
    st->count[cur ^ 1] = 0;
    st->touched_total += count;
    st->c_next = cn;
    st->zc_next = cn >= 0 ? obj[cn] : 0.0;
    st->n_ratio_part = rch;
  }

  // ---- this group's columns, two per step; PIPE issues the next pair's loads
  // before the current pair is computed and stored
  if (lg >= 0) {
    dbl2 scratch[V];
    int a0 = -1, a1 = -1;
    double pa0 = 0.0, pa1 = 0.0;
    bool h0 = cur_l.next(a0, pa0, lane);
    bool h1 = h0 && cur_l.next(a1, pa1, lane);
    dbl2 ta0[V], ta1[V];
    if (h0 && a0 != c) E::load(A + (int64_t)a0 * ld, ta0, ok, base);
    if (h1 && a1 != c) E::load(A + (int64_t)a1 * ld, ta1, ok, base);
    while (h0) {
      int b0 = -1, b1 = -1;
      double pb0 = 0.0, pb1 = 0.0;
      const bool g0 = cur_l.next(b0, pb0, lane);
      const bool g1 = g0 && cur_l.next(b1, pb1, lane);
      dbl2 tb0[V], tb1[V];
      if (PIPE) {
        if (g0 && b0 != c) E::load(A + (int64_t)b0 * ld, tb0, ok, base);
        if (g1 && b1 != c) E::load(A + (int64_t)b1 * ld, tb1, ok, base);
      }
      double* __restrict__ c0 = A + (int64_t)a0 * ld;
      if (a0 == c) E::unit(c0, ok, base, rl);
      else E::update(c0, ta0, f, ok, base, rl, pa0, scratch);
      if (h1) {
        double* __restrict__ c1 = A + (int64_t)a1 * ld;
        if (a1 == c) E::unit(c1, ok, base, rl);
        else E::update(c1, ta1, f, ok, base, rl, pa1, scratch);
      }
      if (!PIPE) {
        if (g0 && b0 != c) E::load(A + (int64_t)b0 * ld, tb0, ok, base);
        if (g1 && b1 != c) E::load(A + (int64_t)b1 * ld, tb1, ok, base);
      }
      a0 = b0;
      a1 = b1;
      pa0 = pb0;
      pa1 = pb1;
      h0 = g0;
      h1 = g1;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        ta0[v] = tb0[v];
        ta1[v] = tb1[v];
      }
    }
  }

  // ---- group 0: columns c' and RHS of this chunk + the next ratio test
  if (g == 0) {
    const int32_t rule = prm->rule;
    const double eps_piv = prm->eps_piv;
    dbl2 nb[V], nc[V];
    {
      double* __restrict__ col = A + rhs * ld;
      const double pj = P[rhs];
      E::load(col, nb, ok, base);
      if (pj != 0.0 || !skip) E::update(col, nb, f, ok, base, rl, pj, nb);
    }
    KeyR k = keyr_none();
    if (cn >= 0) {
      double* __restrict__ col = A + cn * ld;
      const double pj = P[cn];
      E::load(col, nc, ok, base);
      if (pj != 0.0 || !skip) E::update(col, nc, f, ok, base, rl, pj, nc);
      double* __restrict__ Fn = F2 + (cur ^ 1) * ld;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int64_t i = base + (int64_t)v * BLK * 2;
        if (ok[v]) {
          st2<false>(Fn + i, nc[v]);
          ratio_candidate(k, nc[v].x, nb[v].x, row0 + i, basis, rule, eps_piv);
          if (i + 1 < m_local)
            ratio_candidate(k, nc[v].y, nb[v].y, row0 + i + 1, basis, rule, eps_piv);
        }
      }
    }
    k = block_min(k);
    if (threadIdx.x == 0) store_key(ratio_part + chunk, k);
  }
}

// ---------------------------------------------------------------------------
// Utility kernels (outside the pivot loop).
// ---------------------------------------------------------------------------
// out[j] = T[i, j] for one local constraint row (strided gather).
__global__ __launch_bounds__(BLK) void get_row_kernel(const double* __restrict__ A, int64_t ld,
                                                      int64_t N, int64_t i,
                                                      double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  if (j < N) out[j] = A[j * ld + i];
}

// Phase-2 objective row: obj[j] = -cost[j] + sum_i cost[basis[i]] * T[i, j]
// (obj[N-1] = 0 + sum_i cost[basis[i]] * b_i), accumulated in row order i =
// 0..m-1 with a rounded product and a rounded sum per term, skipping rows whose
// basic cost is zero: bit-identical to simplex_amd.lp.phase2_objective and the
// oracle.  One thread per column walks its column contiguously.
__global__ __launch_bounds__(BLK) void phase2_obj_kernel(const double* __restrict__ A,
                                                         int64_t ld, int64_t m, int64_t N,
                                                         const double* __restrict__ cost,
                                                         const int64_t* __restrict__ basis,
                                                         double* __restrict__ obj) {
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  if (j >= N) return;
  double s = (j < N - 1) ? -cost[j] : 0.0;
  const double* __restrict__ col = A + j * ld;
  for (int64_t i = 0; i < m; ++i) {
    const double cb = cost[basis[i]];
    if (cb != 0.0) s = __dadd_rn(s, __dmul_rn(cb, col[i]));
  }
  obj[j] = s;
}

}  // namespace spx
