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

// Diagnostic phase timestamps (tools/probe_phases.py builds a separate library
// with -DSPX_PHASE_TIMING): block 0 / thread 0 of each window kernel records
// s_memrealtime (100 MHz) at its phase boundaries.  Compiled out otherwise.
#ifdef SPX_PHASE_TIMING
__device__ unsigned long long spx_probe_buf[1024 + 2 * 8192];
// flush blocks: [1024 + 2*b] = entry, [1024 + 2*b + 1] = exit of block b
#define SPX_PROBE_BLOCK(which)                                                               \
  do {                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 8192)                                               \
      spx_probe_buf[1024 + 2 * blockIdx.x + (which)] = __builtin_amdgcn_s_memrealtime();    \
  } while (0)
// row_fix blocks: [1024 + 2*(4096 + b) + which]
#define SPX_PROBE_RF_BLOCK(which)                                                            \
  do {                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 4096)                                               \
      spx_probe_buf[1024 + 2 * (4096 + blockIdx.x) + (which)] =                              \
          __builtin_amdgcn_s_memrealtime();                                                  \
  } while (0)
#define SPX_PROBE(slot, kind, phase, cond)                                                  \
  do {                                                                                       \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (cond))                                       \
      spx_probe_buf[(((slot) * 4 + (kind)) * 4 + (phase)) & 1023] =                          \
          __builtin_amdgcn_s_memrealtime();                                                  \
  } while (0)
// flush waves: [2*(4*b + w)] = exit time, [.. + 1] = HW_ID | XCC_ID << 32 | columns << 40
__device__ unsigned long long spx_probe_wave[2 * 4 * 8192];
#define SPX_PROBE_WAVE(w, cols)                                                              \
  do {                                                                                       \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 8192) {                                      \
      unsigned hw_, xc_;                                                                     \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                      \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xc_));                     \
      const int x_ = 2 * (4 * (int)blockIdx.x + (w));                                        \
      spx_probe_wave[x_] = __builtin_amdgcn_s_memrealtime();                                 \
      spx_probe_wave[x_ + 1] = (unsigned long long)hw_ | ((unsigned long long)(xc_ & 0xff) << 32) | \
                               ((unsigned long long)(cols) << 40);                           \
    }                                                                                        \
  } while (0)
#else
#define SPX_PROBE(slot, kind, phase, cond) \
  do {                                     \
  } while (0)
#define SPX_PROBE_BLOCK(which) \
  do {                         \
  } while (0)
#define SPX_PROBE_RF_BLOCK(which) \
  do {                            \
  } while (0)
#define SPX_PROBE_WAVE(w, cols) \
  do {                          \
  } while (0)
#endif

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
  int32_t* nlist;    // 1             : records in `rec` (reset by lazy_ratio slot 0)
  double* rec;       // N x RECW      : the window's touched columns, compacted by the
                     //                 last lazy_norm: [j | path flags, pad, p_0 .. p_{K-1}]
  // Two sets of the per-window buffers (F, P, r, c, made, nlist, rec) alternate
  // by window (the host's parity), so a window's buffers outlive the next
  // window's chain: the row_fix fold resolves window w-1's
  // leaving rows inside window w's chain.  tag, epoch and fix are shared.
  int32_t* fix;      // 5 words: [0..1] G: the window epoch whose leaving rows set s
                     //   still owes (a fold chain's, 0: none); [2..3] Z: the epoch
                     //   a gated row_fix resolved; [4] that kernel's block counter
  int32_t sid;       // this set's index (0 / 1)
  double* frt;       // KW x KW : frt[L*KW + s] = f_s[r_L] for a row whose last leaving
                     //           slot is L (written by a fold chain, for the next one)
  double* Pf;        // KW x N  : p_s[j] at Pf[s*N + j] (slot-major; a fold chain's, for
                     //           the next one)
};

constexpr int RECW = KW + 2;  // doubles per record (272 B)

// Apply pending pivot s to value v at (local row il, column j).
__device__ __forceinline__ double apply_pivot(double v, int64_t il, int64_t j, int64_t rl_s,
                                              int64_t c_s, double f_si, double p_sj,
                                              bool skip) {
  if (j == c_s) return (il == rl_s) ? 1.0 : 0.0;
  if (skip && p_sj == 0.0) return v;
  return (il == rl_s) ? p_sj : msub(v, f_si, p_sj);
}

// This lane's share (keys lane, lane+64, ...) of a per-wave argmin over n >= 1
// keys, in two halves so the loads join the kernel's first batch of
// independent loads: keys_issue() puts up to 8 keys per lane in flight
// (clamped indices: no branch, no loop, nothing for the compiler to sink or
// wait on early); keys_reduce() compares them (and walks any keys beyond 512,
// which only a tableau of more than 32768 columns has).  wave_min() after.
struct Keys8 {
  dbl2 a[8], b[8];  // (v, t) and (row, pad) of keys lane + 64u
};
__device__ __forceinline__ void keys_issue(Keys8& K, const Key* __restrict__ part, int n) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const dbl2* p = reinterpret_cast<const dbl2*>(part + min(lane + 64 * u, n - 1));
    K.a[u] = p[0];
    K.b[u] = p[1];
  }
}
__device__ __forceinline__ KeyR keys_reduce(const Keys8& K, const Key* __restrict__ part, int n) {
  KeyR k = keyr_none();
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (lane + 64 * u < n)
      kmin(k, K.a[u].x, __double_as_longlong(K.a[u].y), __double_as_longlong(K.b[u].x));
  if (n > 512)
    for (int x = lane + 512; x < n; x += 64) kmin(k, part[x].v, part[x].t, part[x].row);
  return k;
}

// Branchless application of pending pivot s to v at (row il, column j): the
// slot's flags are wave-uniform, but a branch would let the compiler sink the
// kernel's early loads below it (one more memory round trip per kernel).
__device__ __forceinline__ double apply_sel(double v, bool il_is_r, bool j_is_c, bool active,
                                            double f, double p, bool skip) {
  const double upd = il_is_r ? p : msub(v, f, p);
  double x = (skip && p == 0.0) ? v : upd;
  x = j_is_c ? (il_is_r ? 1.0 : 0.0) : x;
  return active ? x : v;
}

// v_readlane of an int64 held per lane (lane index wave-uniform).
__device__ __forceinline__ int64_t rdlane64(int64_t v, int lane) {
  const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffff), lane);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), lane);
  return ((int64_t)hi << 32) | (uint32_t)lo;
}

// Fill n keys with "no candidate" (entering partials beyond norm<INIT>'s).
__global__ __launch_bounds__(BLK) void fill_none_kernel(Key* __restrict__ k, int n) {
  const int x = blockIdx.x * BLK + threadIdx.x;
  if (x < n) store_key(k + x, keyr_none());
}

// The start of a pivot call as ONE launch instead of two host copies on the
// stream (each a copy-engine hand-off before the first kernel): the call's
// parameters and the State fields the host sets -- status, forced pivot,
// handshake bound -- plus fill_none_kernel's n keys (windowed calls).
__global__ __launch_bounds__(BLK) void call_begin_kernel(Params* __restrict__ prm, Params p,
                                                         State* __restrict__ st, int32_t status,
                                                         int64_t fc, int64_t fr, int64_t hs,
                                                         Key* __restrict__ k, int n) {
  const int x = blockIdx.x * BLK + threadIdx.x;
  if (x == 0) {
    *prm = p;
    st->status = status;
    st->forced_c = fc;
    st->forced_r = fr;
    st->hs_ticks = hs;
  }
  if (x < n) store_key(k + x, keyr_none());
}

// ---------------------------------------------------------------------------
// lazy_ratio_kernel<KMAX> (slot q < KMAX = number of pending pivots): entering
// column of the coming pivot (or forced), its current values -> F[q], min-ratio
// partials.  grid: ceil(m_local / BLK) blocks, one row per thread.
// Two memory round trips on the critical path: (1) every load that does not
// depend on the column -- entering partials, f_s of this row, the slots'
// (r_s, c_s) lane-indexed, state -- in one batch; (2) after the argmin, the
// stale column c and RHS and their p_s values.  Then stores only.
// ---------------------------------------------------------------------------
template <int KMAX>
__global__ __launch_bounds__(BLK) void lazy_ratio_kernel(
    // the first loads' operands lead the list: they are preloaded into SGPRs
    // (-amdgpu-kernarg-preload-count), so no kernarg fetch precedes them
    const Key* __restrict__ enter_part, State* st, const Params* __restrict__ prm,
    int n_enter_part, int q, const double* __restrict__ A, int64_t ld, int64_t m_local,
    int64_t row0, int64_t N, const double* __restrict__ obj, Window win,
    Key* __restrict__ ratio_part, const int64_t* __restrict__ basis) {
  static_assert(KMAX <= 64, "slots are lane-indexed");
  constexpr int CH = KMAX % 8 == 0 ? 8 : KMAX % 4 == 0 ? 4 : 2;  // slot chunk (divides KMAX)
  SPX_PROBE(q, 0, 0, true);
  const bool block0 = blockIdx.x == 0 && threadIdx.x == 0;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x;
  const bool live = i < m_local;
  const int64_t ic = live ? i : 0;
  // --- batch 1 ---
  Keys8 kk;
  keys_issue(kk, enter_part, n_enter_part);
  // the keys first: loads retire in issue order, and the argmin must not wait
  // for the f_s loads behind them
  asm volatile("" ::: "memory");
  // only the q pending slots, in chunks of 8 behind uniform guards (the
  // guarded loads are still issued together, before the first use)
  double fs[KMAX];
#pragma unroll
  for (int c8 = 0; c8 < KMAX; c8 += CH) {
    if (c8 < q) {
#pragma unroll
      for (int u = 0; u < CH; ++u) fs[c8 + u] = win.F[(int64_t)(c8 + u) * ld + ic];
    } else {
#pragma unroll
      for (int u = 0; u < CH; ++u) fs[c8 + u] = 0.0;
    }
  }
  const int64_t slot_r = win.r[lane < KMAX ? lane : 0];
  const int64_t slot_c = win.c[lane < KMAX ? lane : 0];
  const int32_t status = st->status;
  const int64_t forced_c = st->forced_c;
  const int32_t rule = prm->rule;
  const double eps_piv = prm->eps_piv;
  const bool skip = prm->skip_zero != 0;
  if (q == 0 && block0) {
    // a new window, also when it ends before its first pivot (lazy_norm's
    // compaction and the flush read these later; nothing in this launch does)
    *win.epoch += 1;
    *win.nlist = 0;
  }
  KeyR e = keys_reduce(kk, enter_part, n_enter_part);
#ifdef SPX_PROBE_FINE
  SPX_PROBE(q, 2, 0, e.v != 12345.678);
#endif
  wave_min_dpp(e);
#ifdef SPX_PROBE_FINE
  SPX_PROBE(q, 2, 1, e.v != 12345.678);
#endif
  const bool running = status == ST_RUNNING;
  const int64_t c = (forced_c >= 0) ? forced_c : e.row;
  const bool go = running && c >= 0;  // grid-uniform
  if (block0 && running && c < 0) {
    st->status = ST_OPTIMAL;
    st->c_next = -1;
  }
  SPX_PROBE(q, 0, 1, go);
  // --- batch 2 (c clamped, so the loads are unconditional) ---
  const int64_t cc = go ? c : 0;
  const int64_t rhs = N - 1;
  double fv = A[cc * ld + ic];
  double bv = A[rhs * ld + ic];
  double pc[KMAX], pb[KMAX];
#pragma unroll
  for (int c8 = 0; c8 < KMAX; c8 += CH) {
    if (c8 < q) {
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        pc[c8 + u] = win.P[cc * KW + c8 + u];
        pb[c8 + u] = win.P[rhs * KW + c8 + u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < CH; ++u) pc[c8 + u] = pb[c8 + u] = 0.0;
    }
  }
  const double zc = obj[cc];
  asm volatile("" ::: "memory");  // all loads above are issued before any slot is applied
#pragma unroll
  for (int c8 = 0; c8 < KMAX; c8 += CH) {
    if (c8 < q) {
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int s = c8 + u;
        const bool act = s < q;
        const bool isr = i == rdlane64(slot_r, s) - row0;
        const bool isc = cc == rdlane64(slot_c, s);
        fv = apply_sel(fv, isr, isc, act, fs[s], pc[s], skip);
        bv = apply_sel(bv, isr, false, act, fs[s], pb[s], skip);  // the RHS never enters
      }
    }
  }
  SPX_PROBE(q, 0, 2, fv != 12345.678);
  if (!go) return;
  if (block0) {
    st->c_next = c;
    st->zc_next = zc;
    st->n_ratio_part = gridDim.x * NWAVE;
  }
  KeyR k = keyr_none();
  if (live) {
    win.F[(int64_t)q * ld + i] = fv;
    if (forced_c < 0) ratio_candidate(k, fv, bv, row0 + i, basis, rule, eps_piv);
  }
  if (forced_c < 0) {  // one partial per wave
    wave_min_dpp(k);
    if (lane == 0) store_key(ratio_part + blockIdx.x * NWAVE + (threadIdx.x >> 6), k);
  }
  SPX_PROBE(q, 0, 3, true);
}

// ---------------------------------------------------------------------------
// lazy_norm_kernel<KMAX> (slot q): leaving row, its current values (stale row +
// pending pivots 0..q-1) -> p_q, objective row, column tags, entering partials
// for the next pivot, bookkeeping.  One thread per column; n_ratio = the
// lazy_ratio partial count (a launch constant).  Both lazy kernels reduce and
// publish per WAVE (every wave reduces all partials itself), so neither has a
// block barrier on its critical path.  Round trips as in lazy_ratio: (1) ratio
// partials, this column's objective entry, tag and p_s values, the slots'
// (r_s, c_s), state; (2) after the argmin, the stale row entry and the f_s
// values of the leaving row.  The window's last slot (q == last) compacts the
// touched columns into records for the flush, also when the window stopped.
// ---------------------------------------------------------------------------
template <int KMAX, bool FIN = false>
__global__ __launch_bounds__(BLK) void lazy_norm_kernel(
    const Key* __restrict__ ratio_part, State* st, const Params* __restrict__ prm,
    int n_ratio, int q, const double* __restrict__ A, int64_t ld, int64_t m_local,
    int64_t row0, int64_t N, double* __restrict__ obj, Window win, int last,
    Key* __restrict__ enter_part, int64_t* __restrict__ basis, int64_t* __restrict__ hist,
    const char* __restrict__ gbuf = nullptr, int64_t gstride = 0, int nranks = 0) {
  static_assert(KMAX <= 64, "slots are lane-indexed");
  constexpr int CH = KMAX % 8 == 0 ? 8 : KMAX % 4 == 0 ? 4 : 2;  // slot chunk (divides KMAX)
  const bool block0 = blockIdx.x == 0 && threadIdx.x == 0;
  SPX_PROBE(q, 1, 0, true);
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  const bool live = j < N;
  const int64_t jc = live ? j : 0;
  // --- batch 1 ---
  // FIN (row-sharded, after the all-gather): the keys are the ranks' payload
  // headers, lane-indexed; otherwise this GPU's per-wave ratio partials
  Keys8 kk;
  KeyR gk = keyr_none();
  if constexpr (FIN) {
    if (lane < nranks) {
      const Key* kq = reinterpret_cast<const Key*>(gbuf + lane * gstride);
      gk = KeyR{kq->v, kq->t, kq->row};
    }
  } else {
    keys_issue(kk, ratio_part, n_ratio);
  }
  asm volatile("" ::: "memory");  // the keys first (see lazy_ratio)
  double o = obj[jc];
  const uint32_t old = live ? win.tag[jc] : 0u;
  double ps[KMAX];  // p_s[j] of the q pending slots (chunks of 8, uniform guards)
  const double* __restrict__ Pj = win.P + jc * KW;
#pragma unroll
  for (int c8 = 0; c8 < KMAX; c8 += CH) {
    if (c8 < q) {
#pragma unroll
      for (int u = 0; u < CH; u += 2) {
        const dbl2 pp = ld2<false>(Pj + c8 + u);
        ps[c8 + u] = pp.x;
        ps[c8 + u + 1] = pp.y;
      }
    } else {
#pragma unroll
      for (int u = 0; u < CH; ++u) ps[c8 + u] = 0.0;
    }
  }
  const int64_t slot_r = win.r[lane < KMAX ? lane : 0];
  const int64_t slot_c = win.c[lane < KMAX ? lane : 0];
  const int32_t status = st->status;
  const int64_t c = st->c_next;
  const int64_t forced_r = st->forced_r;
  const int64_t it = st->iters + q;  // iters only changes in the flush
  const double zc = st->zc_next;
  const int64_t hist_cap = st->hist_cap;
  const uint32_t epoch = *win.epoch & TAG_EPOCH;
  const int32_t rule = prm->rule;
  const double eps_opt = prm->eps_opt;
  const int64_t n_enter = prm->n_enter;
  const int64_t iter_limit = prm->iter_limit;
  const bool skip = prm->skip_zero != 0;
  KeyR rk = gk;
  if constexpr (!FIN) rk = keys_reduce(kk, ratio_part, n_ratio);
  wave_min_dpp(rk);
  // FIN: the winning rank (t is unique: exactly one header equals the minimum)
  int wrank = 0;
  if constexpr (FIN) {
    const uint64_t hit = __ballot(lane < nranks && gk.row == rk.row && gk.v == rk.v &&
                                  gk.t == rk.t);
    wrank = hit ? __builtin_ctzll(hit) : 0;
  }
  // stop: no pivot in this slot (grid-uniform)
  bool stop = status != ST_RUNNING;
  int32_t new_status = ST_RUNNING;
  // FIN: a time-limit stop requested through rank 0's payload header
  bool stop_req = false;
  if constexpr (FIN) stop_req = (reinterpret_cast<const Key*>(gbuf)->pad >> 32) != 0;
  if (!stop && (c < 0 || (forced_r < 0 && (it >= iter_limit || stop_req)))) {
    new_status = (c < 0) ? ST_OPTIMAL : ST_LIMIT;
    stop = true;
  }
  const int64_t r = (forced_r >= 0) ? forced_r : rk.row;
  if (!stop && r < 0) {
    new_status = ST_UNBOUNDED;
    stop = true;
  }
  if (block0 && new_status != ST_RUNNING) st->status = new_status;
  if (block0 && stop) win.made[q] = 0;
  SPX_PROBE(q, 1, 1, !stop);
  // --- batch 2 (row clamped, so the loads are unconditional) ---
  // FIN: the winner's normalised row, computed by its owner (lazy_prep_kernel)
  // with this kernel's own formula
  const int64_t rl = (stop || FIN) ? 0 : r - row0;
  double v = 0.0, piv = 1.0, pw = 0.0;
  if constexpr (FIN) {
    pw = reinterpret_cast<const double*>(gbuf + wrank * gstride + PAYLOAD_HDR)[jc];
  } else {
    v = A[jc * ld + rl];
    piv = win.F[(int64_t)q * ld + rl];
  }
  double fr[KMAX];
#pragma unroll
  for (int c8 = 0; c8 < KMAX; c8 += CH) {
    if (!FIN && c8 < q) {
#pragma unroll
      for (int u = 0; u < CH; ++u) fr[c8 + u] = win.F[(int64_t)(c8 + u) * ld + rl];
    } else {
#pragma unroll
      for (int u = 0; u < CH; ++u) fr[c8 + u] = 0.0;
    }
  }
  asm volatile("" ::: "memory");  // all loads above are issued before any slot is applied
  bool zb = false;  // (skip on) some earlier p_s[j] of this window is zero
#pragma unroll
  for (int c8 = 0; c8 < KMAX; c8 += CH) {
    if (c8 < q) {
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int s = c8 + u;
        const bool act = s < q;
        const bool isr = rl == rdlane64(slot_r, s) - row0;
        const bool isc = jc == rdlane64(slot_c, s);
        if constexpr (!FIN) v = apply_sel(v, isr, isc, act, fr[s], ps[s], skip);
        zb |= act && skip && ps[s] == 0.0;
      }
    }
  }
  SPX_PROBE(q, 1, 2, v != 12345.678);
  uint32_t tg = old;  // this column's tag after this slot
  double p = 0.0;
  if (!stop) {
    KeyR ek = keyr_none();
    if (live) {
      p = FIN ? pw : v / piv;
      win.P[j * KW + q] = p;
      const bool nz = (p != 0.0) || !skip;
      if (j == c) {
        o = 0.0;
      } else if (nz) {
        o = msub(o, zc, p);
      }
      obj[j] = o;
      // tag: touched in this window; SPECIAL if it entered, ZERO if (skip on)
      // one of its p_s[j] so far is zero
      const bool tagged = (old & TAG_EPOCH) == epoch;
      if (nz) {
        tg = epoch | ((j == c || (tagged && (old & TAG_SPECIAL))) ? TAG_SPECIAL : 0u) |
             (zb ? TAG_ZERO : 0u);
      } else if (tagged) {
        tg = old | TAG_ZERO;
      }
      if (tg != old) win.tag[j] = tg;
      if (j < n_enter && o < -eps_opt) kmin(ek, (rule == RULE_BLAND) ? 0.0 : o, j, j);
    }
    wave_min_dpp(ek);  // one entering partial per wave
    if (lane == 0) store_key(enter_part + blockIdx.x * NWAVE + (threadIdx.x >> 6), ek);
    if (block0) {
      st->r = r;
      st->c = c;
      st->zc = zc;
      st->piv = piv;
      win.r[q] = r;
      win.c[q] = c;
      win.made[q] = 1;
      basis[r] = c;
      if (it < hist_cap) {
        hist[2 * it] = r;
        hist[2 * it + 1] = c;
      }
    }
  }
  if (q == last) {
    // compact this window's touched columns into records for the flush: wave
    // ballot + LDS prefix over the 4 waves + one atomic per block
    const bool mine = live && (tg & TAG_EPOCH) == epoch;
    __shared__ int wcnt[NWAVE];
    __shared__ int base;
    const uint64_t bal = __ballot(mine);
    const int w = threadIdx.x >> 6;
    if (lane == 0) wcnt[w] = __popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int x = 0; x < NWAVE; ++x) tot += wcnt[x];
      base = tot ? atomicAdd(win.nlist, tot) : 0;
    }
    __syncthreads();
    int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
    for (int x = 0; x < w; ++x) pos += wcnt[x];
    if (mine && pos < N) {  // (pos < N always: one epoch tags each column once)
      double* rc_ = win.rec + (int64_t)pos * RECW;
      reinterpret_cast<int64_t*>(rc_)[0] = j | ((int64_t)(tg >> 30) << 32);
#pragma unroll
      for (int s = 0; s < KMAX; ++s)
        if (s <= q) rc_[2 + s] = (s < q) ? ps[s] : p;
    }
  }
  SPX_PROBE(q, 1, 3, true);
}

// ---------------------------------------------------------------------------
// lazy_prep_kernel<KMAX> (row-sharded rank, slot q): this rank's leaving-row
// candidate -- the argmin of its own ratio partials, or the forced row if it
// owns it -- and that row's CURRENT values (stale row + the pending slots,
// lazy_norm's formula), normalised, as the all-gather payload [key | p[0..N)].
// lazy_norm_kernel<KMAX, true> on every rank then takes the lexicographic
// winner's p: the single-GPU p, bit for bit.  One thread per column.
// ---------------------------------------------------------------------------
template <int KMAX>
__global__ __launch_bounds__(BLK) void lazy_prep_kernel(
    const Key* __restrict__ ratio_part, const State* st, const Params* __restrict__ prm,
    int n_ratio, int q, const double* __restrict__ A, int64_t ld, int64_t m_local,
    int64_t row0, int64_t N, Window win, char* __restrict__ sendbuf, int rank,
    const int32_t* stop_req) {
  static_assert(KMAX <= 64, "slots are lane-indexed");
  constexpr int CH = KMAX % 8 == 0 ? 8 : KMAX % 4 == 0 ? 4 : 2;
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x;
  const bool live = j < N;
  const int64_t jc = live ? j : 0;
  // --- batch 1 ---
  Keys8 kk;
  keys_issue(kk, ratio_part, n_ratio);
  asm volatile("" ::: "memory");
  double ps[KMAX];
  const double* __restrict__ Pj = win.P + jc * KW;
#pragma unroll
  for (int c8 = 0; c8 < KMAX; c8 += CH) {
    if (c8 < q) {
#pragma unroll
      for (int u = 0; u < CH; u += 2) {
        const dbl2 pp = ld2<false>(Pj + c8 + u);
        ps[c8 + u] = pp.x;
        ps[c8 + u + 1] = pp.y;
      }
    } else {
#pragma unroll
      for (int u = 0; u < CH; ++u) ps[c8 + u] = 0.0;
    }
  }
  const int64_t slot_r = win.r[lane < KMAX ? lane : 0];
  const int64_t slot_c = win.c[lane < KMAX ? lane : 0];
  const bool go = st->status == ST_RUNNING && st->c_next >= 0;
  const int64_t forced_r = st->forced_r;
  const bool skip = prm->skip_zero != 0;
  KeyR k = keys_reduce(kk, ratio_part, n_ratio);
  wave_min_dpp(k);
  if (forced_r >= 0)
    k = (forced_r >= row0 && forced_r < row0 + m_local) ? KeyR{0.0, 0, forced_r} : keyr_none();
  const bool have = go && k.row >= 0;  // grid-uniform
  // --- batch 2 (row clamped) ---
  const int64_t rl = have ? k.row - row0 : 0;
  double v = A[jc * ld + rl];
  const double piv = win.F[(int64_t)q * ld + rl];
  double fr[KMAX];
#pragma unroll
  for (int c8 = 0; c8 < KMAX; c8 += CH) {
    if (c8 < q) {
#pragma unroll
      for (int u = 0; u < CH; ++u) fr[c8 + u] = win.F[(int64_t)(c8 + u) * ld + rl];
    } else {
#pragma unroll
      for (int u = 0; u < CH; ++u) fr[c8 + u] = 0.0;
    }
  }
  asm volatile("" ::: "memory");
#pragma unroll
  for (int c8 = 0; c8 < KMAX; c8 += CH) {
    if (c8 < q) {
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int s = c8 + u;
        const bool act = s < q;
        const bool isr = rl == rdlane64(slot_r, s) - row0;
        const bool isc = jc == rdlane64(slot_c, s);
        v = apply_sel(v, isr, isc, act, fr[s], ps[s], skip);
      }
    }
  }
  if (have && live) reinterpret_cast<double*>(sendbuf + PAYLOAD_HDR)[j] = v / piv;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    Key o;
    o.v = have ? k.v : __builtin_inf();
    o.t = have ? k.t : INT64_MAX;
    o.row = have ? k.row : -1;
    o.pad = rank | ((int64_t)stop_requested(rank, stop_req) << 32);  // (spx_kernels.hpp)
    *reinterpret_cast<Key*>(sendbuf) = o;
  }
}

// ---------------------------------------------------------------------------
// flush_lds_kernel<K, D, NTS>: the same update as flush_kernel, over the
// window's compacted records (lazy_norm, last slot), with the column loads
// in flight in LDS instead of VGPRs.  Each wave owns a ring of D 1-KiB LDS
// slots and walks its group's records g, g+G, ... on its own (no block
// barrier): per column one global_load_lds_dwordx4 (128 rows x 8 B) issued D
// columns ahead, one ds_read_b128, the msub chain with p_s[j] in SGPRs (the
// record's p values, loaded one column ahead from an address that depends on
// nothing), one global store.  Per-wave VMEM order is fixed -- one LDS-DMA
// and one store per column (a dummy DMA past the end) -- so a constant
// `s_waitcnt vmcnt(2*(D-1))` retires exactly the slot about to be read.
// Bytes in flight per CU: waves x D KiB (16 x 8 = 128 KiB at K = 16) without
// spending VGPRs on the ring, which the f_s registers (2K per lane) need.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  // M0 = wave-uniform LDS byte base; each lane's 16 B land at base + lane*16
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Record split of flush_lds_kernel: group g takes records g, g+G, g+2G, ...
// (rows of G records, streamed side by side).  A CU's three flush blocks are
// dispatched in three rounds (group-major map: round = 3g / G), and the
// hardware issues from the oldest wave first, so with equal shares the
// third-round blocks ended last and streamed alone
// (profiles/r02/phases_flush_prio.log).  With a tail share x % (fmap bits
// 8-15), the last x % of the record rows go to the first two rounds' groups
// only, still strided: group g takes rows 0..M-1 as before, then (g < Gt =
// 2G/3) records M*G + g, M*G + g + Gt, ...  (Round 5: the tail to the first
// round's groups only was slower at every share, 6-16 %:
// profiles/r05/flush_tail_first_round_sweep.jsonl.)
constexpr int FLUSH_TAIL_DEFAULT = 12;  // profiles/r02/ab/flush_tail_split_ab.jsonl

template <int K, int D, bool NTS, bool PART = false>
__global__ __launch_bounds__(BLK) void flush_lds_kernel(double* __restrict__ A, int64_t ld,
                                                        int64_t m_local, int64_t row0,
                                                        int64_t N, Window win, int npiv,
                                                        int rch, int G,
                                                        const Params* __restrict__ prm,
                                                        State* st, int fmap) {
  static_assert(D >= 2 && D <= 16, "ring depth");
  __shared__ dbl2 ring[NWAVE * D * 64];
  SPX_PROBE(K, 2, 0, true);
  SPX_PROBE_BLOCK(0);
  int nm = 0;  // pivots made in this window: a prefix of its npiv slots
  for (int s = 0; s < npiv; ++s) nm += win.made[s];
  const int L = *win.nlist;
  if (nm == 0) return;
  const bool full = nm == K;
  const bool skip = prm->skip_zero != 0;
  // block -> (row chunk, column group): group-major (consecutive blocks share
  // a group), chunk-major with fmap bit 0; bit 1 rotates the group by the chunk
  int chunk = blockIdx.x % rch, g = blockIdx.x / rch;
  if (fmap & 1) {
    g = blockIdx.x % G;
    chunk = blockIdx.x / G;
  }
  if (fmap & 2) g = (g + chunk) % G;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform, in an SGPR
  if (chunk == 0 && g == 0 && threadIdx.x == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(&st->touched_total), (unsigned long long)L);
    st->iters += nm;
  }
  const int64_t wrow = (int64_t)chunk * 2 * BLK + (int64_t)w * 128;  // this wave's first row
  // this wave's records: g, g+G, ... for rows k < M, then the tail (see above)
  const int tailp = (fmap & 3) == 0 ? (fmap >> 8) & 0xff : 0;
  const int Gt = tailp ? max(1, 2 * G / 3) : G;
  const int M = tailp ? (int)((int64_t)(L / G) * (100 - tailp) / 100) : 0x7fffffff;
  int cnt = g < L ? (L - g + G - 1) / G : 0;
  if (tailp) {
    const int tl = L - M * G;  // tail records, strided over groups 0..Gt-1
    cnt = M + (g < Gt && g < tl ? (tl - g + Gt - 1) / Gt : 0);
  }
  if (wrow >= m_local || cnt <= 0) return;  // wave-uniform: nothing to do
  const int64_t i0 = wrow + 2 * lane;
  const bool ok = i0 < m_local;            // the pair (i0, i0+1) holds local rows
  const int64_t i0c = ok ? i0 : wrow;      // in-column address for idle lanes
  double f[K][2];
#pragma unroll
  for (int s = 0; s < K; ++s) {
    dbl2 fv = dbl2{0.0, 0.0};
    if (s < nm && ok) fv = ld2<false>(win.F + (int64_t)s * ld + i0);
    f[s][0] = fv.x;
    f[s][1] = fv.y;
  }
  // records, r_s and c_s through the constant address space: uniform loads
  // from it are always scalar (SMEM, lgkmcnt), so no VMEM op joins the
  // per-column count below
  typedef const __attribute__((address_space(4))) double cdbl;
  typedef const __attribute__((address_space(4))) int64_t ci64;
  cdbl* rec = (cdbl*)win.rec;
  ci64* hdr = (ci64*)win.rec;
  ci64* wr = (ci64*)win.r;
  ci64* wc = (ci64*)win.c;
  auto rec_of = [&](int k) -> int64_t {
    return (k < M ? g + (int64_t)k * G : (int64_t)M * G + g + (int64_t)(k - M) * Gt) * RECW;
  };
  const uint32_t lds0 =
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) dbl2*)&ring[0]) +
      (uint32_t)(w * D * 64) * (uint32_t)sizeof(dbl2);
  // f must be in registers before the first DMA: the compiler does not see
  // the DMAs, and a wait it placed inside the loop for f would drain them
#pragma unroll
  for (int s = 0; s < K; ++s) asm volatile("" ::"v"(f[s][0]), "v"(f[s][1]));
  wait_vmcnt<0>();
  // prologue: columns 0..D-1 (a dummy re-read of the last real column past cnt)
  const double* last_src = A + (hdr[rec_of(0)] & 0xffffffffll) * ld + i0c;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (d < cnt) last_src = A + (hdr[rec_of(d)] & 0xffffffffll) * ld + i0c;
    glds16(last_src, lds0 + (uint32_t)(d * 64 * sizeof(dbl2)));
  }
  int64_t hn = (D < cnt) ? hdr[rec_of(D)] : 0;  // header of column D (next DMA)
  int64_t hc = hdr[rec_of(0)];                  // header of the column being updated
  // p_s[j] in SGPRs, loaded one column ahead (splitting K = 32 into a half
  // loaded ahead and a half loaded at the column measured 5 % slower)
  double pc[K];
#pragma unroll
  for (int s = 0; s < K; ++s) pc[s] = rec[rec_of(0) + 2 + s];
  const int pq1 = cnt >> 2, pq2 = cnt >> 1, pq3 = cnt - (cnt >> 2);  // quarters of the work
  for (int k = 0; k < cnt; ++k) {
    const int slot = k % D;
    if ((k & 7) == 0) {
      // issue priority by work left: a wave ahead of its CU's others yields
      // issue slots to them (the hardware otherwise prefers the oldest wave,
      // so a CU's first-dispatched block ended ~45 us before its last, which
      // then streamed alone; profiles/r02/phases_flush_waves.log)
      const int rem = cnt - k;
      if (rem > pq3) __builtin_amdgcn_s_setprio(3);
      else if (rem > pq2) __builtin_amdgcn_s_setprio(2);
      else if (rem > pq1) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    // retire column k's DMA: 2 VMEM ops per later column, fewer in the prologue
    if (k >= D - 1) wait_vmcnt<2 * (D - 1)>();
    else wait_vmcnt<D - 1>();
    dbl2 x = ring[(w * D + slot) * 64 + lane];
    auto pv = [&](int s) -> double { return pc[s]; };
    const int64_t j = hc & 0xffffffffll;
    if ((hc >> 32) == 0 && (PART || full)) {
      // fast path: the straight msub chain over the made slots, leaving rows
      // included (row_fix_kernel rewrites those).  PART: the instance launched
      // for a window of fewer than K pivots guards each slot (a separate
      // instance: the guards cost the full-window loop its register budget);
      // a full-size window that stopped early takes the exact path below
      if constexpr (!PART) {
#pragma unroll
        for (int s = 0; s < K; ++s) {
          x.x = msub(x.x, f[s][0], pv(s));
          x.y = msub(x.y, f[s][1], pv(s));
        }
      } else {
#pragma unroll
        for (int s = 0; s < K; ++s) {
          if (s < nm) {
            x.x = msub(x.x, f[s][0], pv(s));
            x.y = msub(x.y, f[s][1], pv(s));
          }
        }
      }
    } else {
      // (r_s, c_s) reloaded on this rare path: the laundered bases keep the
      // compiler from hoisting 2K loop-invariant scalars out of the loop
      ci64* wrk = wr;
      ci64* wck = wc;
      asm volatile("" : "+s"(wrk), "+s"(wck));
#pragma unroll
      for (int s = 0; s < K; ++s) {
        if (s < nm) {
          const int64_t rl = wrk[s] - row0;
          const int64_t cs = wck[s];
          x.x = apply_pivot(x.x, i0, j, rl, cs, f[s][0], pv(s), skip);
          x.y = apply_pivot(x.y, i0 + 1, j, rl, cs, f[s][1], pv(s), skip);
        }
      }
    }
    if (ok) st2<NTS>(A + j * ld + i0, x);
    // DMA of column k + D into the slot just read (its ds_read has retired:
    // x was consumed above); a dummy re-read keeps the VMEM count per column
    if (k + D < cnt) last_src = A + (hn & 0xffffffffll) * ld + i0c;
    glds16(last_src, lds0 + (uint32_t)(slot * 64 * sizeof(dbl2)));
    // next column's header and first p values, and the header of the column
    // after the next DMA: scalar loads issued after this column's ds_read has
    // retired (LDS and SMEM share lgkmcnt), so they land during the next wait
    const int kn = k + 1 < cnt ? k + 1 : k;
    hc = hdr[rec_of(kn)];
#pragma unroll
    for (int s = 0; s < K; ++s) pc[s] = rec[rec_of(kn) + 2 + s];
    hn = (k + D + 1 < cnt) ? hdr[rec_of(k + D + 1)] : 0;
  }
  wait_vmcnt<0>();  // no DMA may land in LDS after the wave has exited
  SPX_PROBE_WAVE(w, cnt);
  SPX_PROBE(K, 2, 1, true);
  SPX_PROBE_BLOCK(1);
}

// ---------------------------------------------------------------------------
// row_fix_kernel<K>: after a window's flush (its made slots: a prefix of K),
// rewrite the leaving rows of the fast-path columns (the window's records
// without SPECIAL / ZERO flags; p values from the records).  For such a column no
// pivot of the window enters it and every p_s[j] != 0, so a leaving row r
// whose last leaving slot is L ends at p_L[j] followed by the later pivots'
// msub updates (their leaving rows differ from r).  One thread per column.
// ---------------------------------------------------------------------------
// fix_rows<K, TPB>: the body of row_fix_kernel -- record kr of `win`, one per
// thread (loaded before the list length is known).  (Round 6's first fold form
// ran this in a loop over records from extra chain blocks; that form lost, and
// the loop with its anti-hoisting index cost the standalone kernel 13.3 -> 15.8
// us per window, so the one-record body is back.)
template <int K, int TPB>
__device__ __forceinline__ void fix_rows(double* A, int64_t ld, int64_t m_local, int64_t row0,
                                         int64_t N, const Window& win, int npiv, int64_t kr) {
  __shared__ double fr[K][K];  // fr[L][s] = f_s[r_L]
  __shared__ int64_t rows[K];
  __shared__ int lastL[K];
  __shared__ int made_sh[K];
  const int t = threadIdx.x;
  // one thread per record of the window (the flush's compacted list: column,
  // path flags, p_0..p_{K-1}).  Two rounds of dependent loads: (1) the record
  // (its index clamped to the buffer, not to the list length, so it does not
  // wait for *nlist), the leaving rows and made flags; (2) the leaving rows' f
  // histories.  (The first form waited for *nlist before the record and
  // loaded f_s[r_L] in a loop of dependent r -> F pairs: 15.1 against 13.9 us.
  // Block-0 stamps, profiles/r05/phases24_rowfix*.log: the kernel starts ~3 us
  // after the flush's last block, then ~2.7 us of loads, ~4 us of msub chains
  // and ~2.5 us to issue the scattered stores (the stores themselves: ~1.4
  // us).  64-thread blocks and the K chains interleaved slot-major measured
  // 14.3-14.9 us, not kept.)
  const int64_t kc = kr < N ? kr : N - 1;  // the record buffer holds N records
  const int nl = *win.nlist;
  const int64_t hdr = reinterpret_cast<const int64_t*>(win.rec)[kc * RECW];
  double p[K];
#pragma unroll
  for (int s = 0; s < K; ++s) p[s] = win.rec[kc * RECW + 2 + s];
  if (t < K) {
    rows[t] = win.r[t] - row0;
    made_sh[t] = t < npiv ? win.made[t] : 0;
  }
  __syncthreads();
  SPX_PROBE(K + 1, 0, 1, hdr != 12345 && p[K - 1] != 12345.678);
  // made slots of this window: a prefix of its npiv launched ones
  int madeK = 0;
#pragma unroll
  for (int s = 0; s < K; ++s) madeK += made_sh[s];
  constexpr int PER = (K * K + TPB - 1) / TPB;
  double fv[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int x = t + u * TPB;
    fv[u] = 0.0;
    if (x < K * K) {
      // (a slot not made in this window holds a stale row: clamped, never used)
      const int64_t rl = min(max(rows[x / K], (int64_t)0), m_local - 1);
      fv[u] = win.F[(int64_t)(x % K) * ld + rl];
    }
  }
  if (t < K) {  // the last leaving slot of row r_t among the made ones
    const int64_t r = rows[t];
    bool last = true;
    for (int s = t + 1; s < madeK; ++s) last &= rows[s] != r;
    lastL[t] = last;
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int x = t + u * TPB;
    if (x < K * K) fr[x / K][x % K] = fv[u];
  }
  SPX_PROBE(K + 1, 0, 2, fv[0] != 12345.678);  // round 2 arrived
  __syncthreads();
  SPX_PROBE(K + 1, 1, 2, true);  // lastL and the barrier done
  const int64_t j = hdr & 0xffffffffll;
  const bool fast = (hdr >> 32) == 0;  // not SPECIAL / ZERO: the flush's plain msub chain
  if (madeK == 0 || kr >= nl || !fast) return;
#pragma unroll
  for (int L = 0; L < K; ++L) {
    if (L >= madeK || !lastL[L] || rows[L] < 0 || rows[L] >= m_local) continue;  // not ours
    double x = p[L];  // p_L[j], then the later slots
#pragma unroll
    for (int s = L + 1; s < K; ++s)
      if (s < madeK) x = msub(x, fr[L][s], p[s]);
    __builtin_nontemporal_store(x, A + j * ld + rows[L]);  // scattered 8-B writes: no L2 allocate
  }
}

// ---------------------------------------------------------------------------
// row_fix_kernel<K>: after a window's flush (its made slots: a prefix of K),
// rewrite the leaving rows of the fast-path columns (the window's records
// without SPECIAL / ZERO flags; p values from the records).  For such a column no
// pivot of the window enters it and every p_s[j] != 0, so a leaving row r
// whose last leaving slot is L ends at p_L[j] followed by the later pivots'
// msub updates (their leaving rows differ from r).  One thread per column.
// ---------------------------------------------------------------------------
template <int K, int TPB = BLK, bool GATED = false>
__global__ __launch_bounds__(TPB) void row_fix_kernel(double* __restrict__ A, int64_t ld,
                                                      int64_t m_local, int64_t row0, int64_t N,
                                                      Window win, int npiv) {
  const int t = threadIdx.x;
  SPX_PROBE(K + 1, 0, 0, true);
  SPX_PROBE_RF_BLOCK(0);
  // GATED (the row_fix fold, DESIGN.md §4b: after the last fold window of a
  // call, or before a window that is not one): this set's leaving rows are
  // rewritten only if a fold chain left them owed (G) and no gated row_fix
  // resolved them since (Z); the last block to pass the gate records Z, so no
  // block of this launch sees its own mark.  Ungated (every window of the
  // launch-per-phase and row-sharded paths): always, and the set owes nothing
  // afterwards (G = 0: nothing of it can be owed to a later fold chain).
  if constexpr (GATED) {
    __shared__ int pend_sh;
    if (t == 0) {
      const int32_t g = win.fix[win.sid], z = win.fix[2 + win.sid];
      pend_sh = g != 0 && g != z;
      __threadfence();
      if (atomicAdd(&win.fix[4], 1) == (int)gridDim.x - 1) {
        win.fix[2 + win.sid] = g;
        win.fix[4] = 0;
      }
    }
    __syncthreads();
    if (!pend_sh) return;
  } else {
    if (blockIdx.x == 0 && t == 0) win.fix[win.sid] = 0;
  }
  fix_rows<K, TPB>(A, ld, m_local, row0, N, win, npiv, (int64_t)blockIdx.x * TPB + t);
#ifdef SPX_PHASE_TIMING
  SPX_PROBE(K + 1, 0, 3, true);  // stores issued
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  SPX_PROBE(K + 1, 1, 0, true);  // stores done
  SPX_PROBE_RF_BLOCK(1);
#endif
}

}  // namespace spx
