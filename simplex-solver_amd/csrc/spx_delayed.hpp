// spx_delayed.hpp — windowed ("delayed") Gauss-Jordan elimination.
//
// The per-element update of pivot s is a function of the element's current
// value, f_s[i] (pivot column before the pivot), p_s[j] (normalised pivot
// row) and (r_s, c_s):
//     j == c_s              -> (i == r_s) ? 1 : 0
//     p_s[j] == 0 (skip on) -> unchanged
//     i == r_s              -> p_s[j]
//     otherwise             -> v - f_s[i] * p_s[j]   (rounded product, rounded difference)
// A window of up to KW pivots is therefore applied to the stored ("stale")
// tableau in ONE streaming pass (flush_kernel), as long as every value a pivot
// needs is produced exactly as the sequential algorithm would produce it:
//   lazy_ratio_kernel : current column c and RHS = stale column + the pending
//                       updates applied in order  -> f_q, ratio partials;
//   lazy_norm_kernel  : current row r = stale row + the pending updates applied
//                       in order -> p_q; objective row (kept current); column
//                       tags; entering partials.
// Each element goes through the identical operation sequence with identical
// operands, so the tableau after the flush is bit-identical to K sequential
// single-pivot eliminations (tests/test_gpu_window.py).  HBM traffic per pivot
// drops from 16 B per touched element to 16 B / K.
//
// Kernel sequence of one window (captured once in a hipGraph):
//   [lazy_ratio(q) -> lazy_norm(q)] for q = 0..K-1, then flush_kernel.
// The slot q is a launch argument (fixed at capture), so no kernel ever
// rewrites a State field that other blocks of the same launch read.  The
// per-pivot critical path is two dependent global round trips per kernel: all
// loads that do not depend on the pivot being chosen (window slots, f_s rows,
// p_s values of this thread's column) are issued before the reduction.
#pragma once
#include "spx_kernels.hpp"

namespace spx {

constexpr int KW = 32;  // window capacity: slots of F / P

// column tags: the window epoch (low 30 bits) + path flags for the flush
constexpr uint32_t TAG_EPOCH = 0x3fffffffu;
constexpr uint32_t TAG_ZERO = 0x40000000u;     // skip on and some p_s[j] == 0: general path
constexpr uint32_t TAG_SPECIAL = 0x80000000u;  // entered in this window: general path

struct Window {
  double* F;         // KW slots x ld : f_s (pivot column before pivot s)
  double* P;         // N x KW        : p_s[j] at P[j*KW + s] (a column's slots contiguous)
  int64_t* r;        // KW            : leaving row (global) of pivot s
  int64_t* c;        // KW            : entering column of pivot s
  int32_t* made;     // KW            : 1 if pivot s of this window was made
  uint32_t* tag;     // N             : epoch (+ flags) of the last window touching column j
  uint32_t* epoch;   // 1             : current window number (bumped by lazy_ratio slot 0)
};

// Apply pending pivot s to value v at (local row il, column j).
__device__ __forceinline__ double apply_pivot(double v, int64_t il, int64_t j, int64_t rl_s,
                                              int64_t c_s, double f_si, double p_sj,
                                              bool skip) {
  if (j == c_s) return (il == rl_s) ? 1.0 : 0.0;
  if (skip && p_sj == 0.0) return v;
  return (il == rl_s) ? p_sj : msub(v, f_si, p_sj);
}

// Fill n keys with "no candidate" (entering partials beyond norm<INIT>'s).
__global__ __launch_bounds__(BLK) void fill_none_kernel(Key* __restrict__ k, int n) {
  const int x = blockIdx.x * BLK + threadIdx.x;
  if (x < n) store_key(k + x, keyr_none());
}

// ---------------------------------------------------------------------------
// lazy_ratio_kernel<KMAX> (slot q < KMAX = number of pending pivots): entering
// column of the coming pivot (or forced), its current values -> F[q], min-ratio
// partials.  grid: ceil(m_local / BLK) blocks, one row per thread.
// ---------------------------------------------------------------------------
template <int KMAX>
__global__ __launch_bounds__(BLK) void lazy_ratio_kernel(
    const double* __restrict__ A, int64_t ld, int64_t m_local, int64_t row0, int64_t N,
    const double* __restrict__ obj, Window win, int q, const Key* __restrict__ enter_part,
    int n_enter_part, Key* __restrict__ ratio_part, const int64_t* __restrict__ basis,
    const Params* __restrict__ prm, State* st) {
  // independent loads first: state, entering partials, this row's f_s
  const int32_t status = st->status;
  const int64_t forced_c = st->forced_c;
  const int32_t rule = prm->rule;
  const double eps_piv = prm->eps_piv;
  const bool skip = prm->skip_zero != 0;
  KeyR e = keyr_none();  // per-wave reduction: no LDS round, no block barrier
  for (int x = threadIdx.x & 63; x < n_enter_part; x += 64)
    kmin(e, enter_part[x].v, enter_part[x].t, enter_part[x].row);
  const int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x;
  const bool live = i < m_local;
  double fs[KMAX];
  int64_t rls[KMAX], cs[KMAX];
#pragma unroll
  for (int s = 0; s < KMAX; ++s) {
    if (s < q) {
      fs[s] = live ? win.F[(int64_t)s * ld + i] : 0.0;
      rls[s] = win.r[s] - row0;
      cs[s] = win.c[s];
    }
  }
  if (status != ST_RUNNING) return;
  int64_t c;
  if (forced_c >= 0) {
    c = forced_c;
  } else {
    wave_min(e);
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
    st->n_ratio_part = gridDim.x * NWAVE;
    if (q == 0) *win.epoch += 1;  // a new window (lazy_norm / flush read it later)
  }
  const int64_t rhs = N - 1;
  double fv = live ? A[c * ld + i] : 0.0;
  double bv = live ? A[rhs * ld + i] : 0.0;
  const double* __restrict__ Pc = win.P + c * KW;
  const double* __restrict__ Pb = win.P + rhs * KW;
#pragma unroll
  for (int s = 0; s < KMAX; ++s) {
    if (s < q) {
      fv = apply_pivot(fv, i, c, rls[s], cs[s], fs[s], Pc[s], skip);
      bv = apply_pivot(bv, i, rhs, rls[s], cs[s], fs[s], Pb[s], skip);
    }
  }
  KeyR k = keyr_none();
  if (live) {
    win.F[(int64_t)q * ld + i] = fv;
    if (forced_c < 0) ratio_candidate(k, fv, bv, row0 + i, basis, rule, eps_piv);
  }
  if (forced_c < 0) {  // one partial per wave
    wave_min(k);
    if ((threadIdx.x & 63) == 0) store_key(ratio_part + blockIdx.x * NWAVE + (threadIdx.x >> 6), k);
  }
}

// ---------------------------------------------------------------------------
// lazy_norm_kernel<KMAX> (slot q): leaving row, its current values (stale row +
// pending pivots 0..q-1) -> p_q, objective row, column tags, entering partials
// for the next pivot, bookkeeping.  One thread per column; n_ratio = the
// lazy_ratio partial count (a launch constant).  Both lazy kernels reduce and
// publish per WAVE (every wave reduces all partials itself), so neither has a
// block barrier on its critical path.
// ---------------------------------------------------------------------------
template <int KMAX>
__global__ __launch_bounds__(BLK) void lazy_norm_kernel(
    const double* __restrict__ A, int64_t ld, int64_t m_local, int64_t row0, int64_t N,
    double* __restrict__ obj, Window win, int q, const Key* __restrict__ ratio_part,
    int n_ratio, Key* __restrict__ enter_part, int64_t* __restrict__ basis,
    int64_t* __restrict__ hist, const Params* __restrict__ prm, State* st) {
  const bool block0 = blockIdx.x == 0 && threadIdx.x == 0;
  // independent loads first
  const int32_t status = st->status;
  const int64_t c = st->c_next;
  const int64_t forced_r = st->forced_r;
  const int64_t it = st->iters + q;  // iters only changes in flush_kernel
  const double zc = st->zc_next;
  const uint32_t epoch = *win.epoch & TAG_EPOCH;
  const int32_t rule = prm->rule;
  const double eps_opt = prm->eps_opt;
  const int64_t n_enter = prm->n_enter;
  const int64_t iter_limit = prm->iter_limit;
  const bool skip = prm->skip_zero != 0;
  KeyR rk = keyr_none();  // per-wave reduction of the per-wave ratio partials
  for (int x = threadIdx.x & 63; x < n_ratio; x += 64)
    kmin(rk, ratio_part[x].v, ratio_part[x].t, ratio_part[x].row);
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  const bool live = j < N;
  double o = live ? obj[j] : 0.0;
  const uint32_t old = live ? win.tag[j] : 0u;
  double ps[KMAX];
  int64_t rls[KMAX], cs[KMAX];
  const double* __restrict__ Pj = win.P + (live ? j : 0) * KW;
#pragma unroll
  for (int s = 0; s < KMAX; ++s) {
    if (s < q) {
      ps[s] = Pj[s];
      rls[s] = win.r[s] - row0;
      cs[s] = win.c[s];
    }
  }
  if (status != ST_RUNNING) {
    if (block0) win.made[q] = 0;
    return;
  }
  if (c < 0 || (forced_r < 0 && it >= iter_limit)) {
    if (block0) {
      st->status = (c < 0) ? ST_OPTIMAL : ST_LIMIT;
      win.made[q] = 0;
    }
    return;
  }
  int64_t r = forced_r;
  if (r < 0) {
    wave_min(rk);
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
  double v = live ? A[j * ld + rl] : 0.0;
  double fr[KMAX];
#pragma unroll
  for (int s = 0; s < KMAX; ++s)
    if (s < q) fr[s] = win.F[(int64_t)s * ld + rl];
#pragma unroll
  for (int s = 0; s < KMAX; ++s)
    if (s < q) v = apply_pivot(v, rl, j, rls[s], cs[s], fr[s], ps[s], skip);
  KeyR ek = keyr_none();
  if (live) {
    const double p = v / piv;
    win.P[j * KW + q] = p;
    const bool nz = (p != 0.0) || !skip;
    if (j == c) {
      o = 0.0;
    } else if (nz) {
      o = msub(o, zc, p);
    }
    obj[j] = o;
    // tag: touched in this window; SPECIAL if it entered, ZERO if (skip on) one
    // of its p_s[j] so far is zero
    const bool tagged = (old & TAG_EPOCH) == epoch;
    bool zb = false;
#pragma unroll
    for (int s = 0; s < KMAX; ++s)
      if (s < q) zb |= skip && ps[s] == 0.0;
    uint32_t nt = old;
    if (nz) {
      nt = epoch | ((j == c || (tagged && (old & TAG_SPECIAL))) ? TAG_SPECIAL : 0u) |
           (zb ? TAG_ZERO : 0u);
    } else if (tagged) {
      nt = old | TAG_ZERO;
    }
    if (nt != old) win.tag[j] = nt;
    if (j < n_enter && o < -eps_opt) kmin(ek, (rule == RULE_BLAND) ? 0.0 : o, j, j);
  }
  wave_min(ek);  // one entering partial per wave
  if ((threadIdx.x & 63) == 0) store_key(enter_part + blockIdx.x * NWAVE + (threadIdx.x >> 6), ek);
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
// flush_kernel<K, NTS>: apply the window's made pivots to every column tagged
// with this window's epoch, one streaming read-modify-write pass.
// grid = rch * G blocks: row chunk of 2*BLK rows (one dbl2 per thread) x G
// column groups; group g owns columns g, g+G, ...  Per batch of BLK columns of
// the group, the block compacts the tagged ones into an LDS list and stages
// their p_s[j] in LDS; every wave then streams the list two columns at a time
// (the next two prefetched), reading p_s[j] as LDS broadcasts.  f_s for the
// thread's two rows stay in registers for the whole launch.
// Fast path (a full window; column not SPECIAL / ZERO): the straight msub
// chain for every row, leaving rows included -- row_fix_kernel then rewrites
// the leaving rows of these columns.  SPECIAL (entered in this window) or ZERO
// (skip on, some p_s[j] == 0) columns and partial windows take the exact
// per-element path (apply_pivot), leaving rows included.
// ---------------------------------------------------------------------------
template <int K, bool NTS>
__global__ __launch_bounds__(BLK) void flush_kernel(double* __restrict__ A, int64_t ld,
                                                    int64_t m_local, int64_t row0, int64_t N,
                                                    Window win, int npiv, int rch, int G,
                                                    const Params* __restrict__ prm, State* st) {
  constexpr int CB = 2;
  __shared__ uint32_t list[BLK];
  __shared__ double pls[BLK * K];
  __shared__ int wcnt[NWAVE];
  int nm = 0;  // pivots made in this window: a prefix of its npiv slots
  for (int s = 0; s < npiv; ++s) nm += win.made[s];
  if (nm == 0) return;
  const bool full = nm == K;
  const uint32_t epoch = *win.epoch & TAG_EPOCH;
  const bool skip = prm->skip_zero != 0;
  const int chunk = blockIdx.x % rch;
  const int g = blockIdx.x / rch;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int64_t i0 = (int64_t)chunk * BLK * 2 + threadIdx.x * 2;
  const bool ok = i0 < m_local;
  double fx[K], fy[K];
#pragma unroll
  for (int s = 0; s < K; ++s) {
    const dbl2 fv = (s < nm && ok) ? ld2<false>(win.F + (int64_t)s * ld + i0) : dbl2{0.0, 0.0};
    fx[s] = fv.x;
    fy[s] = fv.y;
  }
  int64_t touched = 0;
  const int64_t ncol_g = (N - g + G - 1) / G;  // columns g + G*k of this group
  for (int64_t kb = 0; kb < ncol_g; kb += BLK) {
    // 1. compact this batch's tagged columns into the LDS list (entry = k | flags)
    const int64_t k = kb + threadIdx.x;
    const uint32_t tg = (k < ncol_g) ? win.tag[g + k * G] : 0u;
    const bool hit = k < ncol_g && (tg & TAG_EPOCH) == epoch;
    const uint64_t msk = __ballot(hit);
    __syncthreads();  // the previous batch is consumed
    if (lane == 0) wcnt[wid] = __popcll(msk);
    __syncthreads();
    int off = 0, cnt = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) {
      off += (w < wid) ? wcnt[w] : 0;
      cnt += wcnt[w];
    }
    if (hit)
      list[off + __popcll(msk & ((1ull << lane) - 1ull))] =
          (uint32_t)threadIdx.x | (tg & (TAG_SPECIAL | TAG_ZERO));
    __syncthreads();
    // 2. stage p_s[j] of the listed columns: pls[e*K + s]
    for (int x = threadIdx.x; x < cnt * K; x += BLK) {
      const int e = x / K, s = x % K;
      const int64_t j = g + (kb + (int64_t)(list[e] & 0xffffu)) * G;
      pls[x] = win.P[j * KW + s];
    }
    __syncthreads();
    touched += cnt;
    // 3. stream the listed columns, two at a time, the next two prefetched
    dbl2 t[CB];
#pragma unroll
    for (int b = 0; b < CB; ++b)
      if (b < cnt && ok) t[b] = ld2<false>(A + (g + (kb + (int64_t)(list[b] & 0xffffu)) * G) * ld + i0);
    for (int e0 = 0; e0 < cnt; e0 += CB) {
      dbl2 tn[CB];
#pragma unroll
      for (int b = 0; b < CB; ++b) {
        const int e = e0 + CB + b;
        if (e < cnt && ok)
          tn[b] = ld2<false>(A + (g + (kb + (int64_t)(list[e] & 0xffffu)) * G) * ld + i0);
      }
#pragma unroll
      for (int b = 0; b < CB; ++b) {
        const int e = e0 + b;
        if (e < cnt) {
          const uint32_t le = list[e];
          const int64_t j = g + (kb + (int64_t)(le & 0xffffu)) * G;
          const double* __restrict__ pe = pls + e * K;
          dbl2 x = t[b];
          if (full && !(le & (TAG_SPECIAL | TAG_ZERO))) {
#pragma unroll
            for (int s = 0; s < K; ++s) {
              const double p = pe[s];
              x.x = msub(x.x, fx[s], p);
              x.y = msub(x.y, fy[s], p);
            }
          } else {
            for (int s = 0; s < nm; ++s) {
              const int64_t rl = win.r[s] - row0;
              const int64_t cs = win.c[s];
              const double* __restrict__ Fs = win.F + (int64_t)s * ld;
              const double p = pe[s];
              x.x = apply_pivot(x.x, i0, j, rl, cs, ok ? Fs[i0] : 0.0, p, skip);
              x.y = apply_pivot(x.y, i0 + 1, j, rl, cs, ok ? Fs[i0 + 1] : 0.0, p, skip);
            }
          }
          if (ok) st2<NTS>(A + j * ld + i0, x);
        }
      }
#pragma unroll
      for (int b = 0; b < CB; ++b) t[b] = tn[b];
    }
  }
  if (chunk == 0 && threadIdx.x == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(&st->touched_total),
              (unsigned long long)touched);
    if (g == 0) st->iters += nm;
  }
}

// ---------------------------------------------------------------------------
// row_fix_kernel<K>: after a FULL window's flush, rewrite the leaving rows of
// the fast-path columns (tagged, not SPECIAL / ZERO).  For such a column no
// pivot of the window enters it and every p_s[j] != 0, so a leaving row r
// whose last leaving slot is L ends at p_L[j] followed by the later pivots'
// msub updates (their leaving rows differ from r).  One thread per column.
// ---------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(BLK) void row_fix_kernel(double* __restrict__ A, int64_t ld,
                                                      int64_t row0, int64_t N, Window win) {
  int nm = 0;
  for (int s = 0; s < K; ++s) nm += win.made[s];
  if (nm != K) return;
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  if (j >= N) return;
  const uint32_t epoch = *win.epoch & TAG_EPOCH;
  const uint32_t tg = win.tag[j];
  if ((tg & TAG_EPOCH) != epoch || (tg & (TAG_SPECIAL | TAG_ZERO))) return;
  double p[K];
#pragma unroll
  for (int s = 0; s < K; ++s) p[s] = win.P[j * KW + s];
  for (int L = 0; L < K; ++L) {
    const int64_t r = win.r[L];
    bool last = true;
    for (int s = L + 1; s < K; ++s) last &= win.r[s] != r;
    if (!last) continue;
    const int64_t rl = r - row0;
    double x = p[L];
#pragma unroll
    for (int s = 0; s < K; ++s)
      if (s > L) x = msub(x, win.F[(int64_t)s * ld + rl], p[s]);
    A[j * ld + rl] = x;
  }
}

}  // namespace spx
