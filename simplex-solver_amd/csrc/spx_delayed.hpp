// spx_delayed.hpp — windowed ("delayed") Gauss-Jordan elimination.
//
// The per-element update of pivot q is a function of the element's current
// value, f_q[i] (pivot column before the pivot), p_q[j] (normalised pivot
// row) and (r_q, c_q):
//     j == c_q              -> (i == r_q) ? 1 : 0
//     p_q[j] == 0 (skip on) -> unchanged
//     i == r_q              -> p_q[j]
//     otherwise             -> v - f_q[i] * p_q[j]   (rounded product, rounded difference)
// A window of up to KMAX pivots is therefore applied to the stored ("stale")
// tableau in ONE streaming pass per window (flush_kernel), as long as every
// value a pivot needs is produced exactly as the sequential algorithm would:
//   lazy_ratio_kernel : current column c and RHS = stale column + the pending
//                       updates applied in order  -> f, ratio partials;
//   lazy_norm_kernel  : current row r = stale row + the pending updates applied
//                       in order -> p; objective row (kept current); the
//                       window's touched-column list; entering partials.
// Each element goes through the identical operation sequence with identical
// operands, so the tableau after the flush is bit-identical to K sequential
// single-pivot eliminations (tests/test_gpu_engine.py::*window*).  HBM traffic
// per pivot drops from 16 B per touched element to 16 B / K.
//
// Kernel sequence of one window (captured once in a hipGraph):
//   [lazy_ratio(q) -> lazy_norm(q)] for q = 0..K-1, then flush_kernel.
// The slot q is a launch argument (fixed at capture), so no kernel ever
// rewrites a State field that other blocks of the same launch read.
#pragma once
#include "spx_kernels.hpp"

namespace spx {

struct Window {
  double* F;         // KMAX slots x ld  : f_q (pivot column before pivot q)
  double* P;         // KMAX slots x N   : p_q (normalised pivot row)
  int64_t* r;        // KMAX             : leaving row (global) of pivot q
  int64_t* c;        // KMAX             : entering column of pivot q
  int32_t* made;     // KMAX             : 1 if pivot q of this window was made
  uint8_t* touched;  // N                : column already in this window's list
  int* list;         // N                : columns touched in this window
  int* count;        // 1                : list length
};

// Apply pending pivot q to value v at (local row il, column j).
__device__ __forceinline__ double apply_pivot(double v, int64_t il, int64_t j, int64_t rl_q,
                                              int64_t c_q, double f_qi, double p_qj,
                                              bool skip) {
  if (j == c_q) return (il == rl_q) ? 1.0 : 0.0;
  if (skip && p_qj == 0.0) return v;
  return (il == rl_q) ? p_qj : msub(v, f_qi, p_qj);
}

// ---------------------------------------------------------------------------
// lazy_ratio_kernel (slot q = number of pending pivots): entering column of the
// coming pivot (or forced), its current values -> Window.F[q], min-ratio
// partials.  grid: NBr blocks, grid-stride over row pairs.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(BLK) void lazy_ratio_kernel(
    const double* __restrict__ A, int64_t ld, int64_t m_local, int64_t row0, int64_t N,
    const double* __restrict__ obj, Window win, int q, const Key* __restrict__ enter_part,
    int nbn, Key* __restrict__ ratio_part, const int64_t* __restrict__ basis,
    const Params* __restrict__ prm, State* st) {
  if (st->status != ST_RUNNING) return;
  const int32_t rule = prm->rule;
  const double eps_piv = prm->eps_piv;
  const bool skip = prm->skip_zero != 0;
  const int64_t forced_c = st->forced_c;
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
    st->n_ratio_part = gridDim.x;
    if (q == 0) *win.count = 0;  // a new window starts (the flush has read it)
  }
  const int64_t rhs = N - 1;
  const double* __restrict__ colc = A + c * ld;
  const double* __restrict__ colb = A + rhs * ld;
  double* __restrict__ Fq = win.F + (int64_t)q * ld;
  KeyR k = keyr_none();
  const bool forced = forced_c >= 0;
  for (int64_t i = ((int64_t)blockIdx.x * BLK + threadIdx.x) * 2; i < m_local;
       i += (int64_t)gridDim.x * BLK * 2) {
    dbl2 fv = ld2<false>(colc + i);
    dbl2 bv = ld2<false>(colb + i);
    for (int s = 0; s < q; ++s) {
      const int64_t rl = win.r[s] - row0;
      const int64_t cs = win.c[s];
      const double pc = win.P[(int64_t)s * N + c];
      const double pb = win.P[(int64_t)s * N + rhs];
      const dbl2 fs = ld2<false>(win.F + (int64_t)s * ld + i);
      fv.x = apply_pivot(fv.x, i, c, rl, cs, fs.x, pc, skip);
      fv.y = apply_pivot(fv.y, i + 1, c, rl, cs, fs.y, pc, skip);
      bv.x = apply_pivot(bv.x, i, rhs, rl, cs, fs.x, pb, skip);
      bv.y = apply_pivot(bv.y, i + 1, rhs, rl, cs, fs.y, pb, skip);
    }
    st2<false>(Fq + i, fv);
    if (!forced) {
      ratio_candidate(k, fv.x, bv.x, row0 + i, basis, rule, eps_piv);
      if (i + 1 < m_local) ratio_candidate(k, fv.y, bv.y, row0 + i + 1, basis, rule, eps_piv);
    }
  }
  k = block_min(k);
  if (threadIdx.x == 0) store_key(ratio_part + blockIdx.x, k);
}

// ---------------------------------------------------------------------------
// lazy_norm_kernel (slot q): leaving row, its current values (stale row +
// pending pivots 0..q-1) -> p_q, objective row, window list, entering
// partials for the next pivot, bookkeeping.  One thread per column.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(BLK) void lazy_norm_kernel(
    const double* __restrict__ A, int64_t ld, int64_t m_local, int64_t row0, int64_t N,
    double* __restrict__ obj, Window win, int q, const Key* __restrict__ ratio_part,
    Key* __restrict__ enter_part, int64_t* __restrict__ basis, int64_t* __restrict__ hist,
    const Params* __restrict__ prm, State* st) {
  const bool block0 = blockIdx.x == 0 && threadIdx.x == 0;
  if (st->status != ST_RUNNING) {
    if (block0) win.made[q] = 0;
    return;
  }
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  const int32_t rule = prm->rule;
  const double eps_opt = prm->eps_opt;
  const int64_t n_enter = prm->n_enter;
  const bool skip = prm->skip_zero != 0;
  const int64_t it = st->iters + q;  // iters only changes in flush_kernel
  const int64_t c = st->c_next;
  const int64_t forced_r = st->forced_r;
  double o = (j < N) ? obj[j] : 0.0;
  if (c < 0 || (forced_r < 0 && it >= prm->iter_limit)) {
    if (block0) {
      st->status = (c < 0) ? ST_OPTIMAL : ST_LIMIT;
      win.made[q] = 0;
    }
    return;
  }
  int64_t r = forced_r;
  if (r < 0) {
    const KeyR rk = reduce_keys(ratio_part, st->n_ratio_part);
    if (rk.row < 0) {
      if (block0) {
        st->status = ST_UNBOUNDED;
        win.made[q] = 0;
      }
      return;
    }
    r = rk.row;
  }
  const int64_t rl = r - row0;
  const double piv = win.F[(int64_t)q * ld + rl];
  const double zc = st->zc_next;
  bool nz = false;
  KeyR ek = keyr_none();
  if (j < N) {
    double v = A[j * ld + rl];
    for (int s = 0; s < q; ++s) {
      const int64_t rls = win.r[s] - row0;
      v = apply_pivot(v, rl, j, rls, win.c[s], win.F[(int64_t)s * ld + rl],
                      win.P[(int64_t)s * N + j], skip);
    }
    const double p = v / piv;
    win.P[(int64_t)q * N + j] = p;
    nz = (p != 0.0) || !skip;
    if (j == c) {
      o = 0.0;
    } else if (nz) {
      o = msub(o, zc, p);
    }
    obj[j] = o;
    if (j < n_enter && o < -eps_opt) kmin(ek, (rule == RULE_BLAND) ? 0.0 : o, j, j);
  }
  // first touch of a column in this window -> append to the window list
  const bool fresh = nz && !win.touched[j < N ? j : 0] && j < N;
  {
    __shared__ int wcount[NWAVE];
    __shared__ int wbase[NWAVE];
    __shared__ int bbase;
    const unsigned long long mask = __ballot(fresh);
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int wpre = __popcll(mask & ((1ull << lane) - 1ull));
    if (lane == 0) wcount[w] = __popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
      int s = 0;
#pragma unroll
      for (int x = 0; x < NWAVE; ++x) {
        wbase[x] = s;
        s += wcount[x];
      }
      bbase = s ? atomicAdd(win.count, s) : 0;
    }
    __syncthreads();
    if (fresh) {
      win.list[bbase + wbase[w] + wpre] = (int)j;
      win.touched[j] = 1;
    }
  }
  ek = block_min(ek);
  if (threadIdx.x == 0) store_key(enter_part + blockIdx.x, ek);
  if (block0) {
    st->r = r;
    st->c = c;
    st->zc = zc;
    st->piv = piv;
    win.r[q] = r;
    win.c[q] = c;
    win.made[q] = 1;
    basis[r] = c;
    if (it < st->hist_cap) {
      hist[2 * it] = r;
      hist[2 * it + 1] = c;
    }
  }
}

// ---------------------------------------------------------------------------
// flush_kernel: apply the window's pivots (made[0..K)) to every touched
// column, one streaming read-modify-write pass.  grid = rch * G blocks as in
// elim_kernel (row chunk of BLK*R rows, interleaved column groups); each thread
// keeps f_s for its R rows and all KMAX slots in registers; per column the
// KMAX p_s[j] values are uniform (scalar loads).
// ---------------------------------------------------------------------------
template <int R, int KMAX, bool NTS>
__global__ __launch_bounds__(BLK) void flush_kernel(double* __restrict__ A, int64_t ld,
                                                    int64_t m_local, int64_t row0, int64_t N,
                                                    Window win, int npiv, int rch, int G,
                                                    const Params* __restrict__ prm, State* st) {
  constexpr int V = R / 2;
  // pivots made in this window: a prefix of its npiv slots
  int nm = 0;
  for (int s = 0; s < npiv; ++s) nm += win.made[s];
  if (nm == 0) return;
  const int count = *win.count;
  const bool skip = prm->skip_zero != 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->iters += nm;
    st->touched_total += count;
  }
  const int chunk = blockIdx.x % rch;
  const int g = blockIdx.x / rch;
  const int64_t base = (int64_t)chunk * BLK * R + threadIdx.x * 2;
  bool ok[V];
  dbl2 f[KMAX][V];
  int64_t rl[KMAX], cs[KMAX];
#pragma unroll
  for (int s = 0; s < KMAX; ++s) {
    rl[s] = (s < nm) ? win.r[s] - row0 : -1;
    cs[s] = (s < nm) ? win.c[s] : -1;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int64_t i = base + (int64_t)v * BLK * 2;
      ok[v] = i < m_local;
      f[s][v] = (s < nm && ok[v]) ? ld2<false>(win.F + (int64_t)s * ld + i) : dbl2{0.0, 0.0};
    }
  }
  for (int k = g; k < count; k += G) {
    const int64_t j = win.list[k];
    double p[KMAX];
#pragma unroll
    for (int s = 0; s < KMAX; ++s) p[s] = (s < nm) ? win.P[(int64_t)s * N + j] : 0.0;
    double* __restrict__ col = A + j * ld;
    dbl2 t[V];
#pragma unroll
    for (int v = 0; v < V; ++v)
      if (ok[v]) t[v] = ld2<false>(col + base + (int64_t)v * BLK * 2);
#pragma unroll
    for (int s = 0; s < KMAX; ++s) {
      if (s < nm) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const int64_t i = base + (int64_t)v * BLK * 2;
          t[v].x = apply_pivot(t[v].x, i, j, rl[s], cs[s], f[s][v].x, p[s], skip);
          t[v].y = apply_pivot(t[v].y, i + 1, j, rl[s], cs[s], f[s][v].y, p[s], skip);
        }
      }
    }
#pragma unroll
    for (int v = 0; v < V; ++v)
      if (ok[v]) st2<NTS>(col + base + (int64_t)v * BLK * 2, t[v]);
    if (chunk == 0 && threadIdx.x == 0) win.touched[j] = 0;
  }
}

}  // namespace spx
