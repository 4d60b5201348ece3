// spx_kernels.hpp — gfx950 (CDNA4) kernels of the dense simplex pivot engine.
//
// One pivot of the tableau method (the loop inside simple_simplex's
// optimize_json_format, called at reference app/controllers/solver_controller.py:318)
// is three launches on one stream:
//
//   ratio_kernel  : entering column c from the previous pivot's per-block
//                   reduced-cost partials; pivot-column snapshot F = T[:,c];
//                   per-block min-ratio partials over the constraint rows.
//   norm_kernel   : leaving row r from the ratio partials; pivot row
//                   p = T[r,:] / T[r,c]; objective-row update; compaction of
//                   the columns with p[j] != 0; per-block entering partials
//                   for the NEXT pivot; basis / history bookkeeping.
//   elim_kernel   : T[i,j] <- T[i,j] - F[i]*p[j] over the compacted columns,
//                   row r <- p, column c <- e_r.  The HBM-roofline kernel.
//
// Memory layout: the m constraint rows are stored COLUMN-MAJOR
// (column j is ld contiguous doubles), so the ratio test reads two contiguous
// columns, the elimination streams whole columns with 16-B lane accesses, and
// a column whose pivot-row entry is zero is skipped without touching HBM.  The
// objective row lives in its own contiguous vector `obj`.
//
// Arithmetic is fixed to match the oracle bit for bit: IEEE division for p
// and the ratios, separate multiply and subtract (the library is compiled with
// -ffp-contract=off), lexicographic (value, tie) argmin reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spx {

constexpr int BLK = 256;  // threads per workgroup (4 wave64)
constexpr int NWAVE = BLK / 64;

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
  int64_t iter_limit;  // absolute pivot count at which the ratio kernel stops
};

struct State {
  int32_t status;
  int32_t nz_count;       // columns compacted by norm_kernel for this pivot
  int64_t iters;          // pivots since load
  int64_t c;              // entering column of the current pivot
  int64_t r;              // leaving row (global index) of the current pivot
  double zc;              // objective-row entry of column c before the pivot
  double piv;             // pivot element (owner rank only)
  int64_t forced_c;       // >= 0: spx_pivot_at column
  int64_t forced_r;       // >= 0: spx_pivot_at row
  int64_t touched_total;  // sum of nz_count over pivots (byte accounting)
  int64_t hist_cap;
};

// Lexicographic argmin key: smallest v, then smallest t.  `row` carries the
// payload (leaving row / entering column).  t is unique among candidates, so
// every reduction order gives the same answer.
struct Key {
  double v;
  int64_t t;
  int64_t row;
  int64_t pad;
};

__device__ __forceinline__ Key key_none() {
  Key k;
  k.v = __builtin_inf();
  k.t = INT64_MAX;
  k.row = -1;
  k.pad = 0;
  return k;
}

__device__ __forceinline__ bool key_less(const Key& a, const Key& b) {
  return (a.v < b.v) || (a.v == b.v && a.t < b.t);
}

__device__ __forceinline__ Key key_min(const Key& a, const Key& b) { return key_less(b, a) ? b : a; }

__device__ __forceinline__ Key wave_min(Key k) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    Key o;
    o.v = __shfl_xor(k.v, off, 64);
    o.t = __shfl_xor(k.t, off, 64);
    o.row = __shfl_xor(k.row, off, 64);
    o.pad = 0;
    k = key_min(k, o);
  }
  return k;
}

// Block-wide argmin; every thread receives the result.
__device__ __forceinline__ Key block_min(Key k) {
  __shared__ Key sk[NWAVE];
  k = wave_min(k);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sk[w] = k;
  __syncthreads();
  Key r = sk[0];
#pragma unroll
  for (int i = 1; i < NWAVE; ++i) r = key_min(r, sk[i]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ Key reduce_keys(const Key* __restrict__ part, int n) {
  Key k = key_none();
  for (int i = threadIdx.x; i < n; i += BLK) k = key_min(k, part[i]);
  return block_min(k);
}

// Explicit round-to-nearest multiply then subtract: never contracted to FMA.
__device__ __forceinline__ double msub(double t, double f, double p) {
  return __dsub_rn(t, __dmul_rn(f, p));
}

// ---------------------------------------------------------------------------
// ratio_kernel: entering column + pivot-column snapshot + min-ratio partials.
// grid: NBr blocks, grid-stride over row pairs.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(BLK) void ratio_kernel(const double* __restrict__ A, int64_t ld,
                                                    int64_t m_local, int64_t row0, int64_t N,
                                                    const double* __restrict__ obj,
                                                    double* __restrict__ F,
                                                    const Key* __restrict__ enter_part, int nbn,
                                                    Key* __restrict__ ratio_part,
                                                    const int64_t* __restrict__ basis,
                                                    const Params* __restrict__ prm, State* st) {
  if (st->status != ST_RUNNING) return;
  const int32_t rule = prm->rule;
  const double eps_piv = prm->eps_piv;
  const int64_t forced_c = st->forced_c;
  int64_t c;
  if (forced_c >= 0) {
    c = forced_c;
  } else {
    if (st->iters >= prm->iter_limit) {
      if (blockIdx.x == 0 && threadIdx.x == 0) st->status = ST_LIMIT;
      return;
    }
    const Key e = reduce_keys(enter_part, nbn);
    if (e.row < 0) {
      if (blockIdx.x == 0 && threadIdx.x == 0) st->status = ST_OPTIMAL;
      return;
    }
    c = e.row;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->c = c;
    st->zc = obj[c];
    st->nz_count = 0;
  }
  const double* __restrict__ colc = A + c * ld;
  const double* __restrict__ rhs = A + (N - 1) * ld;
  Key k = key_none();
  const bool forced = forced_c >= 0;
  for (int64_t i = ((int64_t)blockIdx.x * BLK + threadIdx.x) * 2; i < m_local;
       i += (int64_t)gridDim.x * BLK * 2) {
    const double2 fv = *reinterpret_cast<const double2*>(colc + i);
    const double2 bv = *reinterpret_cast<const double2*>(rhs + i);
    *reinterpret_cast<double2*>(F + i) = fv;
    if (!forced) {
      if (fv.x > eps_piv) {
        Key q;
        q.v = bv.x / fv.x;
        q.row = row0 + i;
        q.t = (rule == RULE_BLAND) ? basis[row0 + i] : q.row;
        q.pad = 0;
        k = key_min(k, q);
      }
      if (i + 1 < m_local && fv.y > eps_piv) {
        Key q;
        q.v = bv.y / fv.y;
        q.row = row0 + i + 1;
        q.t = (rule == RULE_BLAND) ? basis[row0 + i + 1] : q.row;
        q.pad = 0;
        k = key_min(k, q);
      }
    }
  }
  k = block_min(k);
  if (threadIdx.x == 0) ratio_part[blockIdx.x] = k;
}

// ---------------------------------------------------------------------------
// norm_kernel: one thread per tableau column.
//   MODE_FUSED  (1 rank): leaving row from ratio partials, p, objective,
//                         compaction, entering partials, bookkeeping.
//   MODE_PROW   (sharded, before the p all-reduce): leaving row from the
//                         all-gathered per-rank keys; the owner writes p,
//                         the other ranks write zeros.
//   MODE_FINISH (sharded, after the all-reduce): objective, compaction,
//                         entering partials, bookkeeping.
//   MODE_INIT   entering partials only (after load / objective change).
// ---------------------------------------------------------------------------
constexpr int MODE_FUSED = 0;
constexpr int MODE_PROW = 1;
constexpr int MODE_FINISH = 2;
constexpr int MODE_INIT = 3;

template <int MODE>
__global__ __launch_bounds__(BLK) void norm_kernel(const double* __restrict__ A, int64_t ld,
                                                   int64_t m_local, int64_t row0, int64_t N,
                                                   double* __restrict__ obj,
                                                   const double* __restrict__ F,
                                                   double* __restrict__ P, int* __restrict__ list,
                                                   const Key* __restrict__ keys, int nkeys,
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

  int64_t r = -1;
  if (MODE == MODE_FUSED || MODE == MODE_PROW) {
    r = st->forced_r;
    if (r < 0) {
      const Key rk = reduce_keys(keys, nkeys);
      if (rk.row < 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) st->status = ST_UNBOUNDED;
        return;
      }
      r = rk.row;
    }
  }

  if (MODE == MODE_PROW) {
    const int64_t rl = r - row0;
    if (j < N) {
      double p = 0.0;
      if (rl >= 0 && rl < m_local) p = A[j * ld + rl] / F[rl];
      P[j] = p;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->r = r;
      if (rl >= 0 && rl < m_local) st->piv = F[rl];
    }
    return;
  }

  bool nz = false;
  Key ek = key_none();
  const int64_t c = (MODE == MODE_INIT) ? -1 : st->c;
  if (j < N) {
    double o = obj[j];
    if (MODE != MODE_INIT) {
      double p;
      if (MODE == MODE_FUSED) {
        p = A[j * ld + (r - row0)] / F[r - row0];
        P[j] = p;
      } else {
        p = P[j];
      }
      nz = (p != 0.0) || !skip;
      if (j == c) {
        o = 0.0;
      } else if (nz) {
        o = msub(o, st->zc, p);
      }
      obj[j] = o;
    }
    if (j < n_enter && o < -eps_opt) {
      ek.v = (rule == RULE_BLAND) ? 0.0 : o;
      ek.t = j;
      ek.row = j;
    }
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
      bbase = s ? atomicAdd(&st->nz_count, s) : 0;
    }
    __syncthreads();
    if (nz) list[bbase + wbase[w] + wpre] = (int)j;
  }

  ek = block_min(ek);
  if (threadIdx.x == 0) enter_part[blockIdx.x] = ek;

  if (MODE != MODE_INIT && blockIdx.x == 0 && threadIdx.x == 0) {
    if (MODE == MODE_FUSED) {
      st->r = r;
      st->piv = F[r - row0];
    } else {
      r = st->r;
    }
    basis[r] = c;
    const int64_t it = st->iters;
    if (it < st->hist_cap) {
      hist[2 * it] = r;
      hist[2 * it + 1] = c;
    }
    st->iters = it + 1;
  }
}

// select_kernel (sharded): this rank's best leaving candidate -> sendkey.
__global__ __launch_bounds__(BLK) void select_kernel(const Key* __restrict__ ratio_part, int nbr,
                                                     Key* __restrict__ sendkey, const State* st) {
  const Key k = reduce_keys(ratio_part, nbr);
  if (threadIdx.x == 0) {
    if (st->status == ST_RUNNING) {
      sendkey[0] = k;
    } else {
      sendkey[0] = key_none();
    }
  }
}

// ---------------------------------------------------------------------------
// elim_kernel: the rank-1 Gauss-Jordan update, HBM-bound.
// grid = Rch * G blocks.  Block b owns row chunk (b % Rch) of RC = BLK*R rows
// and column group (b / Rch) of the compacted column list.  Each thread keeps
// its R pivot-column values F[i] in registers for the whole sweep and streams
// R/2 16-B vectors per column, two columns in flight.  NT selects
// non-temporal loads/stores for the once-touched stream.
// ---------------------------------------------------------------------------
typedef double dbl2 __attribute__((ext_vector_type(2)));

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

template <int R, bool NT>
__device__ __forceinline__ void elim_store(double* __restrict__ col, const dbl2 (&t)[R / 2],
                                           const dbl2 (&f)[R / 2], const bool (&ok)[R / 2],
                                           int64_t base, int64_t rl, double pj) {
#pragma unroll
  for (int v = 0; v < R / 2; ++v) {
    const int64_t i = base + (int64_t)v * BLK * 2;
    if (ok[v]) {
      dbl2 o;
      o.x = (i == rl) ? pj : msub(t[v].x, f[v].x, pj);
      o.y = (i + 1 == rl) ? pj : msub(t[v].y, f[v].y, pj);
      st2<NT>(col + i, o);
    }
  }
}

template <int R, bool NT>
__device__ __forceinline__ void elim_unit(double* __restrict__ col, const bool (&ok)[R / 2],
                                          int64_t base, int64_t rl) {
#pragma unroll
  for (int v = 0; v < R / 2; ++v) {
    const int64_t i = base + (int64_t)v * BLK * 2;
    if (ok[v]) {
      dbl2 o;
      o.x = (i == rl) ? 1.0 : 0.0;
      o.y = (i + 1 == rl) ? 1.0 : 0.0;
      st2<NT>(col + i, o);
    }
  }
}

template <int R, bool NT>
__global__ __launch_bounds__(BLK) void elim_kernel(double* __restrict__ A, int64_t ld,
                                                   int64_t m_local, int64_t row0,
                                                   const double* __restrict__ F,
                                                   const double* __restrict__ P,
                                                   const int* __restrict__ list, int rch, int G,
                                                   State* st) {
  static_assert(R % 2 == 0, "R must be even");
  constexpr int V = R / 2;
  if (st->status != ST_RUNNING) return;
  const int count = st->nz_count;
  const int64_t c = st->c;
  const int64_t rl = st->r - row0;
  if (blockIdx.x == 0 && threadIdx.x == 0) st->touched_total += count;
  const int chunk = blockIdx.x % rch;
  const int g = blockIdx.x / rch;
  const int kb = (int)(((int64_t)g * count) / G);
  const int ke = (int)(((int64_t)(g + 1) * count) / G);
  if (kb >= ke) return;

  const int64_t base = (int64_t)chunk * BLK * R + threadIdx.x * 2;
  dbl2 f[V];
  bool ok[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int64_t i = base + (int64_t)v * BLK * 2;
    ok[v] = i < m_local;
    f[v] = ok[v] ? *reinterpret_cast<const dbl2*>(F + i) : dbl2{0.0, 0.0};
  }

  int k = kb;
  for (; k + 1 < ke; k += 2) {
    const int j0 = list[k];
    const int j1 = list[k + 1];
    const double p0 = P[j0];
    const double p1 = P[j1];
    double* __restrict__ c0 = A + (int64_t)j0 * ld;
    double* __restrict__ c1 = A + (int64_t)j1 * ld;
    dbl2 t0[V], t1[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int64_t i = base + (int64_t)v * BLK * 2;
      if (ok[v]) {
        t0[v] = ld2<NT>(c0 + i);
        t1[v] = ld2<NT>(c1 + i);
      }
    }
    if (j0 == c) elim_unit<R, NT>(c0, ok, base, rl);
    else elim_store<R, NT>(c0, t0, f, ok, base, rl, p0);
    if (j1 == c) elim_unit<R, NT>(c1, ok, base, rl);
    else elim_store<R, NT>(c1, t1, f, ok, base, rl, p1);
  }
  if (k < ke) {
    const int j0 = list[k];
    const double p0 = P[j0];
    double* __restrict__ c0 = A + (int64_t)j0 * ld;
    if (j0 == c) {
      elim_unit<R, NT>(c0, ok, base, rl);
    } else {
      dbl2 t0[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int64_t i = base + (int64_t)v * BLK * 2;
        if (ok[v]) t0[v] = ld2<NT>(c0 + i);
      }
      elim_store<R, NT>(c0, t0, f, ok, base, rl, p0);
    }
  }
}

// Sum of nranks P buffers (in-process virtual ranks; RCCL does this across
// processes).  Only one rank holds nonzeros, so the sum is exact.
__global__ __launch_bounds__(BLK) void sum_rows_kernel(double* const* __restrict__ srcs,
                                                       int nsrc, double* __restrict__ dst,
                                                       int64_t n) {
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int q = 0; q < nsrc; ++q) s += srcs[q][j];
  dst[j] = s;
}

}  // namespace spx
