// spx_chain.hpp — the pivot chain of one window as ONE persistent launch.
//
// The windowed path (spx_delayed.hpp) chooses each pivot with two dependent
// launches, lazy_ratio -> lazy_norm, so every pivot pays two kernel
// boundaries and two re-reads of partials that another XCD wrote before the
// boundary (~62 % of a pivot at K = 24).  chain_kernel runs all
// K pivots of a window in one launch of B co-resident blocks (one per CU) that
// hand the two all-to-all reductions of a pivot to each other in-launch:
//
//   ratio phase q : entering column c_q = winner of the blocks' entering
//                   records; each block rebuilds column c_q and the RHS on its
//                   rows (stale + pending slots), stores f_q, and publishes its
//                   best (ratio, tie, row, pivot element) record;
//   norm phase q  : leaving row r_q = winner of the ratio records; each block
//                   rebuilds row r_q on its columns, p_q = row / pivot element,
//                   updates the objective row and tags, and publishes its best
//                   entering candidate for pivot q+1.
//
// The arithmetic is lazy_ratio's / lazy_norm's, operation for operation (the
// same apply_sel chain over the pending slots in slot order, the same IEEE
// divisions), so the window's f_s, p_s, objective row, basis and records are
// bit-identical to the launch-per-phase chain, and the flush that follows is
// unchanged.  What changes is only where each value lives between pivots:
//   * a thread owns one column j and one row i of its block's ranges for the
//     whole window: p_s[j], f_s[i], the current RHS of row i, basis[i],
//     obj[j] and tag[j] stay in its registers;
//   * the only cross-block data are the per-block records (8-byte tagged
//     granules {tag, 32-bit value}, one sc1 store each: the data is the flag)
//     and the two history vectors another block needs: P[c][0..q) (the
//     entering column's p values, owner -> every ratio phase) and F[0..q)[r]
//     (the leaving row's f values, owner -> every norm phase).  Those are
//     stored sc1 (write-through) and drained (s_waitcnt vmcnt(0)) by every
//     storing wave before its block's record is stored, and read with sc1
//     loads after the record poll matched (MI355X_MICROARCH.md, visibility
//     table row 1; cdna_hip_programming.md Guideline 16 R1/R2);
//   * the stale tableau A is not written during the launch: plain loads.
// Every spin is bounded: a block that waits ~4 s for a record stores
// ST_FAULT and exits, so the grid always drains (the host reports the fault).
// Record tags are unique per (window epoch, slot, phase), so records of an
// earlier window never match; one buffer per phase kind suffices because no
// block can publish phase q+1's records before every block consumed phase q's.
#pragma once
#include "spx_delayed.hpp"

namespace spx {

#ifdef SPX_PHASE_TIMING
// per-block chain timestamps (tools/probe_phases.py --blocks,
// tools/probe_stragglers.py): [q][event][block], events 0 ratio record stored,
// 1 ratio poll done, 2 entering record stored, 3 entering poll done (of slot
// q+1's ratio phase), 4 / 5 the ratio / norm phase's dependent loads arrived,
// 6 / 7 their pending slots applied; spx_probe_chain_hw[block] = HW_ID |
// XCC_ID << 32 of the block's CU
constexpr int PROBE_CHAIN_EV = 8;
__device__ unsigned long long spx_probe_chain[32 * PROBE_CHAIN_EV * 256];
__device__ unsigned long long spx_probe_chain_hw[256];
#define SPX_PROBE_CHAIN_R(role, q, ev)                                                     \
  do {                                                                                    \
    if (threadIdx.x == 0 && (role) < 256 && (q) < 32)                                     \
      spx_probe_chain[((q) * PROBE_CHAIN_EV + (ev)) * 256 + (role)] =                     \
          __builtin_amdgcn_s_memrealtime();                                               \
  } while (0)
#define SPX_PROBE_CHAIN(q, ev) SPX_PROBE_CHAIN_R(blockIdx.x, q, ev)
// stamped by thread 0 once `cond` (a value of the awaited data) is known
#define SPX_PROBE_CHAIN_T(q, ev, cond)                                                     \
  do {                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < 256 && (q) < 32 && (cond))                       \
      spx_probe_chain[((q) * PROBE_CHAIN_EV + (ev)) * 256 + blockIdx.x] =                 \
          __builtin_amdgcn_s_memrealtime();                                               \
  } while (0)
#define SPX_PROBE_CHAIN_HW()                                                               \
  do {                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < 256) {                                           \
      unsigned hw_, xc_;                                                                  \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                   \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xc_));                  \
      spx_probe_chain_hw[blockIdx.x] = (unsigned long long)hw_ | ((unsigned long long)xc_ << 32); \
    }                                                                                     \
  } while (0)
#else
#define SPX_PROBE_CHAIN(q, ev) \
  do {                         \
  } while (0)
#define SPX_PROBE_CHAIN_R(role, q, ev) \
  do {                                 \
  } while (0)
#define SPX_PROBE_CHAIN_T(q, ev, cond) \
  do {                                 \
  } while (0)
#define SPX_PROBE_CHAIN_HW() \
  do {                       \
  } while (0)
#endif

constexpr int32_t ST_FAULT = 5;       // a chain exchange timed out (never on a healthy GPU)
constexpr int32_t ST_NOTRES = 6;      // a chain's blocks were not all resident: its window did not run
// Records are stored granule-major: granule g of block b at rec[g * CHAIN_MAX_BLOCKS + b],
// so one poll instruction of a wave reads 64 blocks' granule g as 512 contiguous bytes.
// A record is a polled header plus extras that only the winner's record is read for
// (after the poll, beside the phase's other dependent loads): the winning row's or
// column's whole window history, so no other history is ever stored write-through.
constexpr int ENTER_HDR = 3;            // o_lo, o_hi, j
constexpr int ENTER_REC = ENTER_HDR + 2 * 32;  // + p_0..p_q[j] (lo, hi each)
constexpr int RATIO_HDR = 4;            // v_lo, v_hi, row, t (t read under Bland only)
constexpr int RATIO_REC = RATIO_HDR + 2 + 2 * 32;  // + RHS of row (lo, hi), f_0..f_q[row]
constexpr int CHAIN_MAX_BLOCKS = 256;   // one block per CU
constexpr unsigned CHAIN_SPIN_MAX = 1u << 22;
// Row-sharded chain (chain_shard_kernel): the ratio
// records of every rank's blocks land in every rank's buffer, at block slot
// rank * B + b of planes CHAIN_SH_SLOTS apart; two halves by pivot parity, then
// one plane of window-end granules.
constexpr int CHAIN_MAX_RANKS = 16;
constexpr int CHAIN_SH_SLOTS = 512;     // nranks x B ratio records (8 per polling lane)
constexpr int CHAIN_SH_PLANES = 2 * RATIO_REC + 1;
// Start handshake planes (chain_start): one arrival granule per block, then
// the verdict word (slot 0 of the next plane).  Single GPU: after the ratio
// records of gr_ratio; row shards: after CHAIN_SH_PLANES, in the buffer of the
// rank that leads the caller's device group.
constexpr int HS_PLANE_1GPU = RATIO_REC;
constexpr int HS_PLANE_SHARD = CHAIN_SH_PLANES;
// Row shards, after the handshake planes: one plane of IPC release marks
// (spx_capi.hip close_peers: slot q = rank q's mapping of this buffer is
// closed, value = the import generation), then the owner-push inbox.
constexpr int CLOSE_PLANE_SHARD = HS_PLANE_SHARD + 2;
constexpr int INBOX_PLANE_SHARD = HS_PLANE_SHARD + 3;
// Owner-push inbox (round 5): the leaving row's stale values,
// pushed by its owner into every peer's buffer as tagged granules: [half by
// pivot parity][low word, high word][column], each plane inbox_stride(N)
// granules.
__host__ __device__ constexpr int64_t inbox_stride(int64_t N) { return (N + 63) / 64 * 64; }
__host__ __device__ constexpr int64_t shard_record_granules(int64_t N) {
  return (int64_t)INBOX_PLANE_SHARD * CHAIN_SH_SLOTS + 4 * inbox_stride(N);
}

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

// Granule store / load: agent scope on one GPU; system scope (SYS) for the
// sharded chain's records, which peers on other GPUs write over xGMI
template <bool SYS = false>
__device__ __forceinline__ void g_store(gu64* g, unsigned tag, unsigned val) {
  __hip_atomic_store(g, ((unsigned long long)tag << 32) | val, __ATOMIC_RELAXED,
                     SYS ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT);
}
template <bool SYS = false>
__device__ __forceinline__ unsigned long long g_load(const gu64* g) {
  return __hip_atomic_load(const_cast<gu64*>(g), __ATOMIC_RELAXED,
                           SYS ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT);
}

// The row-sharded chain's view of the other ranks (a kernel argument): their
// ratio-record buffers and stale tableaux (peer pointers: IPC-mapped across
// processes, plain device pointers between the virtual ranks of one process).
struct ChainPeers {
  int rank, nranks;
  unsigned long long* ratio[CHAIN_MAX_RANKS];  // (CHAIN_SH_PLANES + 2) x CHAIN_SH_SLOTS granules each
  const double* A[CHAIN_MAX_RANKS];
  int64_t ld[CHAIN_MAX_RANKS];
  int64_t row0[CHAIN_MAX_RANKS];
  const int32_t* stop_req;  // rank 0: the host's time-limit stop request (pinned)
  // leaving-row transport: 0 pull (every rank reads the owner's tableau
  // through a peer pointer), 1 owner-push (the owner writes the row into every
  // peer's inbox); agreed by every rank at import
  int push;
  // device groups (ranks sharing a GPU) for the start handshake: group g's
  // lowest rank gleader[g] holds its arrival plane and verdict word; gmask[g]
  // has a bit per member rank; `group` is this rank's
  int ngroups, group;
  int gleader[CHAIN_MAX_RANKS];
  uint32_t gmask[CHAIN_MAX_RANKS];
};
// write-through (sc1) store / load of one double
__device__ __forceinline__ void wt_store(double* p, double v) {
  __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double wt_load(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64*)const_cast<double*>(p), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// granule kinds
constexpr int GK_RATIO = 0;  // ratio record of slot q
constexpr int GK_ENTER = 1;  // entering record published by slot q (for slot q+1)
constexpr int GK_DONE = 2;   // sharded: a block's last row gather of the window returned
// granule tag: never 0 (the buffers start zeroed), unique per (epoch, slot, kind)
__device__ __forceinline__ unsigned rec_tag(uint32_t epoch, int q, int kind) {
  return 0x80000000u | ((epoch & 0x7fffffu) << 8) | ((unsigned)q << 2) | (unsigned)kind;
}
// a double as two granules (low word, high word) at g[0], g[stride]
__device__ __forceinline__ void g_store_d(gu64* g, unsigned tag, double v, int stride = 1) {
  const unsigned long long x = (unsigned long long)__double_as_longlong(v);
  g_store(g, tag, (unsigned)x);
  g_store(g + stride, tag, (unsigned)(x >> 32));
}
__device__ __forceinline__ double g_decode_d(unsigned long long lo, unsigned long long hi) {
  return __longlong_as_double((long long)((lo & 0xffffffffull) | (hi << 32)));
}

// argmin key + two doubles of payload, lexicographic on (v, t) as kmin
struct KeyP {
  double v;
  int64_t t;
  int64_t row;
  double a, b;
};
__device__ __forceinline__ KeyP keyp_none() {
  return KeyP{__builtin_inf(), INT64_MAX, -1, 0.0, 0.0};
}
__device__ __forceinline__ void kmin2(KeyP& k, double v, int64_t t, int64_t row, double a,
                                      double b) {
  const bool take = (v < k.v) || (v == k.v && t < k.t);
  k.v = take ? v : k.v;
  k.t = take ? t : k.t;
  k.row = take ? row : k.row;
  k.a = take ? a : k.a;
  k.b = take ? b : k.b;
}
__device__ __forceinline__ double dbits(int64_t x) { return __longlong_as_double(x); }
__device__ __forceinline__ int64_t ibits(double x) { return __double_as_longlong(x); }
template <int CTRL>
__device__ __forceinline__ void kmin2_dpp(KeyP& k) {
  kmin2(k, dbits(dpp64<CTRL>(ibits(k.v))), dpp64<CTRL>(k.t), dpp64<CTRL>(k.row),
        dbits(dpp64<CTRL>(ibits(k.a))), dbits(dpp64<CTRL>(ibits(k.b))));
}
template <int D>
__device__ __forceinline__ void kmin2_swap(KeyP& k) {
  kmin2(k, dbits(swap64<D>(ibits(k.v))), swap64<D>(k.t), swap64<D>(k.row),
        dbits(swap64<D>(ibits(k.a))), dbits(swap64<D>(ibits(k.b))));
}
// every lane receives the wave's winner and its payload
__device__ __forceinline__ void wave_min2(KeyP& k) {
  kmin2_dpp<0x128>(k);  // row_ror:8
  kmin2_dpp<0x124>(k);  // row_ror:4
  kmin2_dpp<0x4E>(k);   // quad_perm [2,3,0,1]
  kmin2_dpp<0xB1>(k);   // quad_perm [1,0,3,2]
  kmin2_swap<16>(k);
  kmin2_swap<32>(k);
}
// Wave argmin of (v, t), lexicographic, by value first: a DPP min of v, then
// the lanes holding it by ballot.  When t grows with the lane index among the
// lanes (t_mono) the lowest such lane wins; otherwise a DPP min of t among the
// tied lanes picks it.  Returns the winning lane (wave-uniform) or -1 when no
// lane is valid.  About a fifth of wave_min2's instructions.
template <int CTRL>
__device__ __forceinline__ double dpp_minf(double x) {
  return fmin(x, dbits(dpp64<CTRL>(ibits(x))));
}
template <int D>
__device__ __forceinline__ double swap_minf(double x) {
  return fmin(x, dbits(swap64<D>(ibits(x))));
}
__device__ __forceinline__ double wave_minf(double x) {
  x = dpp_minf<0x128>(x);
  x = dpp_minf<0x124>(x);
  x = dpp_minf<0x4E>(x);
  x = dpp_minf<0xB1>(x);
  x = swap_minf<16>(x);
  return swap_minf<32>(x);
}
template <int CTRL>
__device__ __forceinline__ int64_t dpp_mini(int64_t x) {
  const int64_t y = dpp64<CTRL>(x);
  return y < x ? y : x;
}
template <int D>
__device__ __forceinline__ int64_t swap_mini(int64_t x) {
  const int64_t y = swap64<D>(x);
  return y < x ? y : x;
}
__device__ __forceinline__ int wave_argmin(double v, int64_t t, bool valid, bool t_mono) {
  const double vmin = wave_minf(valid ? v : __builtin_inf());
  uint64_t tie = __ballot(valid && v == vmin);
  if (tie == 0ull) return -1;
  if (!t_mono && __popcll(tie) > 1) {
    int64_t x = ((tie >> (threadIdx.x & 63)) & 1ull) ? t : INT64_MAX;
    x = dpp_mini<0x128>(x);
    x = dpp_mini<0x124>(x);
    x = dpp_mini<0x4E>(x);
    x = dpp_mini<0xB1>(x);
    x = swap_mini<16>(x);
    x = swap_mini<32>(x);
    tie = __ballot(((tie >> (threadIdx.x & 63)) & 1ull) && t == x);
  }
  return (int)__builtin_ctzll(tie);
}
// the winning lane's key and payload, to every lane
__device__ __forceinline__ KeyP key_of_lane(const KeyP& k, int ln) {
  if (ln < 0) return keyp_none();
  return KeyP{rdlane(k.v, ln), rdlane64(k.t, ln), rdlane64(k.row, ln), rdlane(k.a, ln),
              rdlane(k.b, ln)};
}

// The block's key from its 4 wave keys (lanes 0..3 hold them, lexicographic
// (v, t) as kmin2): a quad DPP min of v, the tied lanes by ballot, and --
// unless t grows with the lane (mono) -- a quad DPP min of t among them; then
// the winner's fields read once.  Fewer dependent steps than two kmin2_dpp
// rounds (10 DPP moves and a branchy compare each) plus key_of_lane.
__device__ __forceinline__ KeyP block_key4(const KeyP& mine, bool mono) {
  const int lane = threadIdx.x & 63;
  double m = mine.v;
  m = dpp_minf<0xB1>(m);  // quad_perm [1,0,3,2]
  m = dpp_minf<0x4E>(m);  // quad_perm [2,3,0,1]
  const double vmin = rdlane(m, 0);
  uint64_t tie = __ballot(lane < 4 && mine.v == vmin) & 0xfull;
  if (!mono && __popcll(tie) > 1) {
    int64_t x = ((tie >> lane) & 1ull) ? mine.t : INT64_MAX;
    x = dpp_mini<0xB1>(x);
    x = dpp_mini<0x4E>(x);
    const int64_t tmin = rdlane64(x, 0);
    tie &= __ballot(((tie >> lane) & 1ull) && mine.t == tmin);
  }
  return key_of_lane(mine, tie ? (int)__builtin_ctzll(tie) : 0);
}

// Bounded spin bookkeeping: true (and ST_FAULT stored) once a wait ran too long.
__device__ __forceinline__ bool spin_fail(unsigned& spins, State* st) {
  if (++spins < CHAIN_SPIN_MAX) {
    __builtin_amdgcn_s_sleep(1);
    return false;
  }
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_store((gu32*)&st->status, (unsigned)ST_FAULT, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

constexpr int GK_START = 3;  // a block's arrival at the start handshake (chain_start)

// Start handshake of a persistent chain launch ("Residency").
// The chain's exchanges need every block of the launch resident at once; a
// block that is not (its CU held by another kernel, another chain queued in
// front of it on the same hardware queue) would leave the others spinning.
// Before its first store every block stores an arrival granule (tag: window
// epoch W, kind GK_START), and wave 0 polls its device group's arrivals for
// at most `bound` ticks of s_memrealtime (100 MHz).  The outcome is fixed ONCE
// per group and window by a compare-and-swap on the group's verdict word,
// from the value of an earlier window to (W, GO) -- every arrival seen -- or
// (W, ABORT) -- the wait ran out: the first CAS wins and every block, late
// ones included, reads the same verdict.  So either every block runs the
// window or none stores anything; on ABORT the host reruns the window
// (ST_NOTRES).  A verdict word already past W means W was aborted (no group
// runs a later window before every group finished W).  Row shards with several
// device groups also wait for every group's verdict: the window runs only
// when all said GO.  Returns 0 go, 1 abort, 2 fault (a group never decided
// within ~4 s).  Wave 0 only: the caller hands the result to its block.
// a - b of two window epochs (TAG_EPOCH: 30 bits, wrapping), sign-extended
__device__ __forceinline__ int32_t epoch_diff(uint32_t a, uint32_t b) {
  return (int32_t)((a - b) << 2) >> 2;
}

template <bool SYS>
__device__ __forceinline__ int chain_start(const gu64* arr, int nslots, int B, uint32_t gmask,
                                           gu64* vword, uint32_t W, int64_t bound,
                                           uint64_t t0, const ChainPeers* pe, State* st) {
  const int lane = threadIdx.x & 63;
  const unsigned tag = rec_tag(W, 0, GK_START);
  // a negative bound -k forces ABORT of every k-th window epoch (k = 1: every
  // window; the rerun test hooks); the others wait the automatic bound
  bool late = bound < 0 && (W % (uint32_t)(-bound)) == 0u;
  if (bound < 0) bound = SYS ? 10000000 : 2000;
  for (unsigned spins = 0; !late;) {
    bool ok = true;
    for (int x = lane; x < nslots; x += 64)
      if ((gmask >> (x / B)) & 1u) ok &= (unsigned)(g_load<SYS>(arr + x) >> 32) == tag;
    // (read with the arrivals) the group's verdict word: once it holds W or a
    // later window, W is decided, so stop waiting.  A rank that reruns late
    // -- its host drained after its peers' -- then walks through the windows
    // its peers aborted without waiting out the bound for each, and catches
    // up with them (tests/test_gpu_peer_chain.py, --late-drain)
    const unsigned long long vw0 = g_load<SYS>(vword);
    if (__all(ok)) break;
    if (epoch_diff((uint32_t)(vw0 >> 8), W) >= 0) break;
    late = (int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > bound;
    if (!late && spin_fail(spins, st)) return 2;
  }
  unsigned v = 0u;
  if (lane == 0) {
    const unsigned long long want = ((unsigned long long)W << 8) | (late ? 2u : 1u);
    unsigned long long cur = g_load<SYS>(vword);
    for (;;) {
      const int32_t d = epoch_diff((uint32_t)(cur >> 8), W);
      if (d > 0) {  // the group is past W: W was aborted
        cur = 2u;
        break;
      }
      if (d == 0) break;  // decided by another block
      if (__hip_atomic_compare_exchange_strong(vword, &cur, want, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED,
                                               SYS ? __HIP_MEMORY_SCOPE_SYSTEM
                                                   : __HIP_MEMORY_SCOPE_AGENT)) {
        cur = want;
        break;
      }
    }
    v = (unsigned)(cur & 0xffu);
  }
  v = __shfl(v, 0, 64);
  if (v != 1u) return 1;
  if (pe == nullptr || pe->ngroups <= 1) return 0;
  // every other device group's verdict (system-scope loads of their words).
  // A group still undecided once the handshake bound has passed is decided
  // for it: ABORT(W) by a compare-and-swap from its older word (round 6; the
  // first CAS on a word wins, its own blocks included, so every group reads
  // the same outcome), and every group reruns the window -- instead of the
  // ~4 s spin ending in ST_FAULT when a peer's host drained late.
  const int64_t gbound = bound < 0 ? 10000000 : bound;
  for (unsigned spins = 0;;) {
    bool dec = true, ab = false;
    if (lane < pe->ngroups) {
      gu64* w = (gu64*)pe->ratio[pe->gleader[lane]] + (size_t)(HS_PLANE_SHARD + 1) * CHAIN_SH_SLOTS;
      unsigned long long x = g_load<true>(w);
      int32_t d = epoch_diff((uint32_t)(x >> 8), W);
      if (d < 0 && (int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > gbound) {
        const unsigned long long want = ((unsigned long long)W << 8) | 2u;
        if (__hip_atomic_compare_exchange_strong(w, &x, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM))
          x = want;
        d = epoch_diff((uint32_t)(x >> 8), W);
      }
      dec = d >= 0;
      ab = d > 0 || (d == 0 && (x & 0xffu) == 2u);
    }
    if (__any(ab)) return 1;
    if (__all(dec)) return 0;
    if (spin_fail(spins, st)) return 2;
  }
}

// Poll the B record headers of one phase (lane l reads blocks l, l+64, ...)
// until every tag matches; reduce the keys over the wave.  The key's payload
// `a` is the entering record's objective entry (z_c); `b` the winning block.
// Returns false on timeout (ST_FAULT stored).  RATIO selects the record kind,
// G the header granules read (3, or 4 for Bland's ratio records).
template <bool RATIO>
__device__ __forceinline__ void decode_record(KeyP& k, const unsigned long long (&g)[4], int b,
                                              int rule, unsigned& stop) {
  const double v = g_decode_d(g[0], g[1]);
  const unsigned idx = (unsigned)g[2];
  // granule 3 of a ratio record: t (bits 0-30) and the sharded chain's stop
  // request (bit 31; rank 0's blocks)
  if (RATIO) stop |= (unsigned)g[3] >> 31;
  if (idx == 0xffffffffu) return;
  if constexpr (RATIO) {
    // Dantzig ties go to the lowest row (t = row); Bland's to the lowest
    // basic-variable index (granule 3)
    kmin2(k, v, rule == RULE_BLAND ? (int64_t)((unsigned)g[3] & 0x7fffffffu) : (int64_t)idx,
          (int64_t)idx, 0.0, (double)b);
  } else {
    // Dantzig: most negative reduced cost; Bland: lowest index (key 0)
    kmin2(k, rule == RULE_BLAND ? 0.0 : v, (int64_t)idx, (int64_t)idx, v, (double)b);
  }
}

template <bool RATIO, int G, int RPL, bool SYS, int rs>
__device__ __forceinline__ bool poll_records_n(const gu64* recs, int B, unsigned tag,
                                               int rule, KeyP& k, State* st, bool* stop) {
  const int lane = threadIdx.x & 63;
  // lane l reads blocks l, l+64, ... (RPL records): every load of a pass is
  // issued before the first tag check, so a pass is one round trip (one pass
  // in flight: more passes measured slower, tools/chain_probe.hip)
  for (unsigned spins = 0;;) {
    unsigned long long g[RPL][4];
#pragma unroll
    for (int x = 0; x < RPL; ++x) {
      const int b = min(lane + 64 * x, B - 1);  // clamped: no branch around the loads
#pragma unroll
      for (int u = 0; u < 4; ++u)
        g[x][u] = u < G ? g_load<SYS>(recs + (size_t)u * rs + b)
                        : (unsigned long long)tag << 32;
    }
    bool ok = true;
#pragma unroll
    for (int x = 0; x < RPL; ++x)
#pragma unroll
      for (int u = 0; u < 4; ++u) ok &= (unsigned)(g[x][u] >> 32) == tag;
    if (__all(ok)) {
      k = keyp_none();
      unsigned sb = 0u;
#pragma unroll
      for (int x = 0; x < RPL; ++x)
        if (lane + 64 * x < B) decode_record<RATIO>(k, g[x], lane + 64 * x, rule, sb);
      if (stop) *stop = __ballot(sb != 0u) != 0ull;
      break;
    }
    if (spin_fail(spins, st)) return false;
  }
  // one record per lane: lane order is block order, and a block's rows and
  // columns all precede the next block's, so t grows with the lane except for
  // Bland's ratio key (a basic-variable index)
  const bool mono = RPL == 1 && !(RATIO && rule == RULE_BLAND);
  k = key_of_lane(k, wave_argmin(k.v, k.t, k.row >= 0, mono));
  asm volatile("" ::: "memory");  // the loads that follow must not be hoisted above the poll
  return true;
}

template <bool RATIO, int G, bool SYS = false, int rs = CHAIN_MAX_BLOCKS>
__device__ __forceinline__ bool poll_records(const gu64* recs, int B, unsigned tag,
                                             int rule, KeyP& k, State* st,
                                             bool* stop = nullptr) {
  if (B <= 64) return poll_records_n<RATIO, G, 1, SYS, rs>(recs, B, tag, rule, k, st, stop);
  if (B <= 128) return poll_records_n<RATIO, G, 2, SYS, rs>(recs, B, tag, rule, k, st, stop);
  if (!SYS || B <= 256)
    return poll_records_n<RATIO, G, 4, SYS, rs>(recs, B, tag, rule, k, st, stop);
  return poll_records_n<RATIO, G, 8, SYS, rs>(recs, B, tag, rule, k, st, stop);
}

// The dependent loads of a phase from the winning record (block wb): lane
// s < n reads the history pair at planes h0 + 2s, h0 + 2s + 1, and every lane
// reads NE wave-uniform pairs at planes e0 + 2x.  One pass re-reads until every
// granule carries the record's tag.  Returns false on timeout.
template <int NE, bool SYS = false, int rs = CHAIN_MAX_BLOCKS>
__device__ __forceinline__ bool load_extras(const gu64* rec, int wb, int h0, int n, int e0,
                                            unsigned tag, double& hv, double (&ev)[2],
                                            State* st) {
  const int lane = threadIdx.x & 63;
  const bool mine = lane < n;
  const gu64* g = rec + (size_t)(h0 + 2 * (mine ? lane : 0)) * rs + wb;
  const gu64* e = rec + (size_t)e0 * rs + wb;
  for (unsigned spins = 0;;) {
    const unsigned long long lo = g_load<SYS>(g), hi = g_load<SYS>(g + rs);
    unsigned long long x[2 * NE > 0 ? 2 * NE : 1];
#pragma unroll
    for (int u = 0; u < 2 * NE; ++u) x[u] = g_load<SYS>(e + (size_t)u * rs);
    bool good = !mine || ((unsigned)(lo >> 32) == tag && (unsigned)(hi >> 32) == tag);
#pragma unroll
    for (int u = 0; u < 2 * NE; ++u) good &= (unsigned)(x[u] >> 32) == tag;
    if (__all(good)) {
      hv = mine ? g_decode_d(lo, hi) : 0.0;
#pragma unroll
      for (int u = 0; u < NE; ++u) ev[u] = g_decode_d(x[2 * u], x[2 * u + 1]);
      return true;
    }
    if (spin_fail(spins, st)) return false;
  }
}

// Publish a block's record: the wave keys are in sk[], and hist(ww, idx, s)
// returns slot s of the history of the winner idx of wave ww (s = 33: the
// RATIO extra, the row's RHS); after the block barrier wave 0 reduces the NW
// keys (every lane the same winner), its lanes store the winner's extras, then
// lane 0 the header (program order: the extras leave first).  RATIO: header v,
// row, t; extras [extra, history].
template <int NW, bool RATIO, bool SYS = false, int rs = CHAIN_MAX_BLOCKS, typename Dst, typename Hist>
__device__ __forceinline__ void publish_record(Dst dst, int nd, unsigned tag, int nh,
                                               const KeyP (&sk)[NW], Hist hist,
                                               unsigned stopbit = 0u, bool mono = false) {
  const int lane = threadIdx.x & 63;
  KeyP k;
  if constexpr (NW == 4) {
    // one LDS read (lane x < 4 takes wave x's key), a quad DPP min and the
    // tied lanes by ballot (block_key4; as publish_local)
    k = block_key4(lane < NW ? sk[lane] : keyp_none(), mono);
  } else {
    k = sk[0];
#pragma unroll
    for (int x = 1; x < NW; ++x) kmin2(k, sk[x].v, sk[x].t, sk[x].row, sk[x].a, sk[x].b);
  }
  const int ww = (int)k.b;  // the winning wave (a payload slot of the block key)
  const bool none = k.row < 0;
  constexpr int H0 = RATIO ? RATIO_HDR + 2 : ENTER_HDR;  // first history plane
  // this lane's granule (the same for every destination): lane x < 2*nh
  // history granule x; RATIO: lanes 62, 63 the extra (row's RHS)
  // (lanes 62, 63 may store both: slot 31's history and the extra)
  int plane = -1, plane2 = -1;
  unsigned val = 0u, val2 = 0u;
  if (!none) {
    if (lane < 2 * nh) {
      const unsigned long long x =
          (unsigned long long)__double_as_longlong(hist(ww, k.row, lane >> 1));
      plane = H0 + lane;
      val = (lane & 1) ? (unsigned)(x >> 32) : (unsigned)x;
    }
    if (RATIO && lane >= 62) {
      const unsigned long long x =
          (unsigned long long)__double_as_longlong(hist(ww, k.row, 33));
      plane2 = RATIO_HDR + (lane - 62);
      val2 = (lane & 1) ? (unsigned)(x >> 32) : (unsigned)x;
    }
  }
  const unsigned long long vb = (unsigned long long)__double_as_longlong(RATIO ? k.v : k.a);
  // (granule 3: t, and the stop request in bit 31)
  const unsigned g3 = (none ? 0x7fffffffu : (unsigned)k.t) | (stopbit << 31);
  for (int d = 0; d < nd; ++d) {  // every destination (one GPU: nd = 1)
    gu64* rb = dst(d);
    if (plane >= 0) g_store<SYS>(rb + (size_t)plane * rs, tag, val);
    if (RATIO && plane2 >= 0) g_store<SYS>(rb + (size_t)plane2 * rs, tag, val2);
    if (lane == 0) {
      g_store<SYS>(rb + 0 * rs, tag, (unsigned)vb);
      g_store<SYS>(rb + 1 * rs, tag, (unsigned)(vb >> 32));
      g_store<SYS>(rb + 2 * rs, tag, none ? 0xffffffffu : (unsigned)k.row);
      if (RATIO) g_store<SYS>(rb + 3 * (size_t)rs, tag, g3);
    }
  }
}

// The single-GPU form of publish_record: one destination, no stop bit.  (The
// shard form's destination loop and stop bit, compiled out for one
// destination, still measured 0.1-0.3 us per pivot slower inside chain_kernel:
// profiles/r03/ab_chain_regression_bisect.jsonl.)
// (pq: the slot, for the probe build's stamps inside the publish; blockIdx 0)
#if defined(SPX_PHASE_TIMING) && defined(SPX_PROBE_FINE)
#define SPX_PROBE_PUB(pq, ph, cond) SPX_PROBE((pq) + 32, RATIO ? 0 : 1, ph, cond)
#else
#define SPX_PROBE_PUB(pq, ph, cond) \
  do {                              \
  } while (0)
#endif
template <int NW, bool RATIO, typename Hist>
__device__ __forceinline__ void publish_local(gu64* rec, int b, unsigned tag, int nh,
                                              const KeyP (&sk)[NW], Hist hist, int pq = 0,
                                              bool mono = false) {
  (void)pq;
  const int lane = threadIdx.x & 63;
  KeyP k;
  if constexpr (NW == 4) {
    // one LDS read (lane x < 4 takes wave x's key), a quad DPP min of the
    // values and the tied lanes by ballot (mono: t grows with the wave);
    // two full kmin2_dpp rounds measured 0.13 us per pivot slower
    // (profiles/r04/ab_block_key4.jsonl)
    k = block_key4(lane < NW ? sk[lane] : keyp_none(), mono);
  } else if constexpr (NW == 8) {
    // lanes 0..7 hold the wave keys: the row-of-16 DPP reduction (rotations
    // by 8 and 4, then the quad steps) leaves lane 0 with their minimum
    k = lane < NW ? sk[lane] : keyp_none();
    kmin2_dpp<0x128>(k);  // row_ror:8
    kmin2_dpp<0x124>(k);  // row_ror:4
    kmin2_dpp<0x4E>(k);   // quad_perm [2,3,0,1]
    kmin2_dpp<0xB1>(k);   // quad_perm [1,0,3,2]
    k = key_of_lane(k, 0);
  } else {
    k = sk[0];
#pragma unroll
    for (int x = 1; x < NW; ++x) kmin2(k, sk[x].v, sk[x].t, sk[x].row, sk[x].a, sk[x].b);
  }
  const int ww = (int)k.b;  // the winning wave (a payload slot of the block key)
  const bool none = k.row < 0;
  SPX_PROBE_PUB(pq, 0, k.v != 12345.678);  // block key reduced
  gu64* rb = rec + b;
  constexpr int H0 = RATIO ? RATIO_HDR + 2 : ENTER_HDR;  // first history plane
  if (!none) {
    // lane x < 2*nh: history granule x; RATIO: lanes 62, 63 the extra (row's RHS)
    if (lane < 2 * nh) {
      const unsigned long long x =
          (unsigned long long)__double_as_longlong(hist(ww, k.row, lane >> 1));
      SPX_PROBE_PUB(pq, 1, x != 12345ull);  // history read from LDS
      g_store(rb + (size_t)(H0 + lane) * CHAIN_MAX_BLOCKS, tag,
                    (lane & 1) ? (unsigned)(x >> 32) : (unsigned)x);
    }
    if (RATIO && lane >= 62) {
      const unsigned long long x =
          (unsigned long long)__double_as_longlong(hist(ww, k.row, 33));
      g_store(rb + (size_t)(RATIO_HDR + (lane - 62)) * CHAIN_MAX_BLOCKS, tag,
                    (lane & 1) ? (unsigned)(x >> 32) : (unsigned)x);
    }
  }
  if (lane == 0) {
    const unsigned long long vb = (unsigned long long)__double_as_longlong(RATIO ? k.v : k.a);
    g_store(rb + 0 * CHAIN_MAX_BLOCKS, tag, (unsigned)vb);
    g_store(rb + 1 * CHAIN_MAX_BLOCKS, tag, (unsigned)(vb >> 32));
    g_store(rb + 2 * CHAIN_MAX_BLOCKS, tag, none ? 0xffffffffu : (unsigned)k.row);
    if (RATIO)
      g_store(rb + 3 * CHAIN_MAX_BLOCKS, tag, none ? 0xffffffffu : (unsigned)k.t);
  }
  SPX_PROBE_PUB(pq, 2, true);  // every store issued
}

// system-scope load of one double (the sharded chain's row gather from a peer)
__device__ __forceinline__ double sys_load(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(
      (gu64*)const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

// The pending slots 0..q-1 of a window applied to one stale value, as masks
// ("Slot application as masks"; LEAN: slots >= q are exact
// identities on +0 histories), shared by chain_kernel and chain_shard_kernel
// (one implementation of each phase's slot chain; forceinline, so each kernel
// compiles the same code as when the loops were written out in it).
// ratio_slots: column c on my row `row` (its f history fs, lane s of pcl =
// p_s[c]; rmask: slots my row left at).
template <int KMAX, int CH, bool LEAN>
__device__ __forceinline__ double ratio_slots(double fv, const double (&fs)[KMAX], double pcl,
                                              uint32_t rmask, int q, int64_t row, int64_t c,
                                              int64_t slot_r, int64_t slot_c, bool skip) {
  const int lane = threadIdx.x & 63;
  const uint32_t qm = (1u << q) - 1u;
  if (__ballot(lane < q && (slot_c == c || (skip && pcl == 0.0))) == 0ull) {
    if (__ballot((rmask & qm) != 0u) == 0ull) {
#pragma unroll
      for (int c8 = 0; c8 < KMAX; c8 += CH) {
        if (c8 < q) {
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            const int s = c8 + u;
            const double x = msub(fv, fs[s], rdlane(pcl, s));
            if constexpr (LEAN) fv = x;  // (s >= q: +0 histories, an identity)
            else fv = s < q ? x : fv;
          }
        }
      }
    } else {
#pragma unroll
      for (int c8 = 0; c8 < KMAX; c8 += CH) {
        if (c8 < q) {
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            const int s = c8 + u;
            const double p_s = rdlane(pcl, s);
            double x = msub(fv, fs[s], p_s);
            x = ((rmask >> s) & 1u) ? p_s : x;  // (bit s >= q is never set)
            if constexpr (LEAN) fv = x;
            else fv = s < q ? x : fv;
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int c8 = 0; c8 < KMAX; c8 += CH) {
      if (c8 < q) {
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int s = c8 + u;
          const bool act = s < q;
          const bool isr = row == rdlane64(slot_r, s);
          const bool isc = c == rdlane64(slot_c, s);
          fv = apply_sel(fv, isr, isc, act, fs[s], rdlane(pcl, s), skip);
        }
      }
    }
  }
  return fv;
}
// norm_slots: row r on my column jc (its p history ps, lane s of frl = f_s[r],
// lane q the pivot element; zmask / cmask: slots whose p_s[jc] was 0 under the
// skip rule / that entered jc).
template <int KMAX, int CH, bool LEAN>
__device__ __forceinline__ double norm_slots(double v, const double (&ps)[KMAX], double frl,
                                             uint32_t zmask, uint32_t cmask, int q, bool jlive,
                                             int64_t r, int64_t jc, int64_t slot_r,
                                             int64_t slot_c, bool skip) {
  const int lane = threadIdx.x & 63;
  const uint32_t qmn = (1u << q) - 1u;
  const double frm = LEAN ? (lane < q ? frl : 0.0) : frl;
  if (__ballot(lane < q && slot_r == r) == 0ull) {
    if (__ballot(jlive && ((zmask | cmask) & qmn) != 0u) == 0ull) {
#pragma unroll
      for (int c8 = 0; c8 < KMAX; c8 += CH) {
        if (c8 < q) {
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            const int s = c8 + u;
            const double x = msub(v, rdlane(frm, s), ps[s]);
            if constexpr (LEAN) v = x;  // (s >= q: +0 histories, an identity)
            else v = s < q ? x : v;
          }
        }
      }
    } else {
#pragma unroll
      for (int c8 = 0; c8 < KMAX; c8 += CH) {
        if (c8 < q) {
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            const int s = c8 + u;
            double x = msub(v, rdlane(frm, s), ps[s]);
            x = ((zmask >> s) & 1u) ? v : x;  // (bits s >= q are never set)
            x = ((cmask >> s) & 1u) ? 0.0 : x;
            if constexpr (LEAN) v = x;
            else v = s < q ? x : v;
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int c8 = 0; c8 < KMAX; c8 += CH) {
      if (c8 < q) {
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int s = c8 + u;
          const bool act = s < q;
          const bool isr = r == rdlane64(slot_r, s);
          const bool isc = jc == rdlane64(slot_c, s);
          v = apply_sel(v, isr, isc, act, rdlane(frl, s), ps[s], skip);
        }
      }
    }
  }
  return v;
}

// The norm phase's update of my column at slot q (lazy_norm's arithmetic):
// p_q = v / piv, the skip / entered masks, the objective entry, the column
// tag and the entering key for pivot q+1; the RHS column (xown) the same with
// p = prhs (p_q[rhs]).  Shared by both chain kernels (forceinline).
template <int KMAX, bool LH>
__device__ __forceinline__ void norm_update(KeyP& ek, double& pq, double (&ps)[KMAX],
                                            uint32_t& zmask, uint32_t& cmask, double& o,
                                            uint32_t& tg, bool jlive, int64_t j, int64_t c, int q,
                                            double v, double piv, double zc, bool skip, bool zb,
                                            uint32_t W, int64_t n_enter, double eps_opt,
                                            int32_t rule, bool xown, uint32_t& zmx, double& ox,
                                            uint32_t& tgx, double prhs, uint32_t qmn,
                                            double* pxl) {
  ek = keyp_none();
  pq = 0.0;
  if (jlive) {
    const double p = v / piv;
    pq = p;
    zmask |= (skip && p == 0.0) ? (1u << q) : 0u;
    cmask |= (j == c) ? (1u << q) : 0u;
    if constexpr (!LH) {
#pragma unroll
      for (int s = 0; s < KMAX; ++s) ps[s] = (s == q) ? p : ps[s];
    }
    const bool nz = (p != 0.0) || !skip;
    if (j == c) {
      o = 0.0;
    } else if (nz) {
      o = msub(o, zc, p);
    }
    const bool tagged = (tg & TAG_EPOCH) == W;
    if (nz) {
      tg = W | ((j == c || (tagged && (tg & TAG_SPECIAL))) ? TAG_SPECIAL : 0u) |
           (zb ? TAG_ZERO : 0u);
    } else if (tagged) {
      tg = tg | TAG_ZERO;
    }
    // key (o, j) under Dantzig, (0, j) under Bland; payload o (z_c)
    if (j < n_enter && o < -eps_opt) kmin2(ek, rule == RULE_BLAND ? 0.0 : o, j, j, o, 0.0);
  }
  if (xown) {  // the RHS column: the same update with p = p_q[rhs] (never j == c)
    const bool zbx = (zmx & qmn) != 0u;
    zmx |= (skip && prhs == 0.0) ? (1u << q) : 0u;
    const bool nz = (prhs != 0.0) || !skip;
    if (nz) ox = msub(ox, zc, prhs);
    const bool tagged = (tgx & TAG_EPOCH) == W;
    if (nz) {
      tgx = W | ((tagged && (tgx & TAG_SPECIAL)) ? TAG_SPECIAL : 0u) | (zbx ? TAG_ZERO : 0u);
    } else if (tagged) {
      tgx = tgx | TAG_ZERO;
    }
    pxl[q] = prhs;
  }
}

// The window's touched columns compacted into the flush's records (as
// lazy_norm's last slot): wave ballot + LDS prefix + one atomic per block;
// the RHS column (xown) follows its wave's own columns.  pget(s) = my column's
// p_s.  Shared by both chain kernels (forceinline).
template <int KMAX, int NW, typename PGet>
__device__ __forceinline__ void compact_records(const Window& win, int64_t N, int q, uint32_t W,
                                                bool jlive, bool xown, int64_t j, uint32_t tg,
                                                uint32_t tgx, const double* pxl, int t, int lane,
                                                int w, int* wcnt, int& base, PGet pget) {
  const bool mine = jlive && (tg & TAG_EPOCH) == W;
  const bool minex = xown && (tgx & TAG_EPOCH) == W;
  const uint64_t bal = __ballot(mine);
  const uint64_t balx = __ballot(minex);
  if (lane == 0) wcnt[w] = __popcll(bal) + __popcll(balx);
  __syncthreads();
  if (t == 0) {
    int tot = 0;
    for (int x = 0; x < NW; ++x) tot += wcnt[x];
    base = tot ? (int)__hip_atomic_fetch_add((gu32*)win.nlist, (unsigned)tot, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)
               : 0;
  }
  __syncthreads();
  int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
  for (int x = 0; x < w; ++x) pos += wcnt[x];
  if (mine && pos < N) {
    double* rc_ = win.rec + (int64_t)pos * RECW;
    reinterpret_cast<int64_t*>(rc_)[0] = j | ((int64_t)(tg >> 30) << 32);
#pragma unroll
    for (int s = 0; s < KMAX; ++s)
      if (s < q) rc_[2 + s] = pget(s);
  }
  if (minex) {
    const int px = pos - __popcll(bal & ((1ull << lane) - 1ull)) + __popcll(bal);
    if (px < N) {
      double* rc_ = win.rec + (int64_t)px * RECW;
      reinterpret_cast<int64_t*>(rc_)[0] = (N - 1) | ((int64_t)(tgx >> 30) << 32);
#pragma unroll
      for (int s = 0; s < KMAX; ++s)
        if (s < q) rc_[2 + s] = pxl[s];
    }
  }
}

// ---------------------------------------------------------------------------
// chain_kernel<KMAX, CB>: the pivots of one window (npiv <= KMAX slots) on one
// GPU.  grid = B blocks of CB threads (one block per CU, every block
// resident); block b owns columns [b*cpb, ...) and rows [b*rpb, ...),
// cpb, rpb <= CB, one of each per thread.  Wave 0 of a block polls the record
// headers and hands the winner to the block through LDS; every thread then
// loads what its column / row needs (the winning record's history beside the
// stale tableau value).  n_ep / enter_part: pivot 0's entering partials,
// written by the previous kernel (norm<INIT> or the previous window's chain);
// the chain writes one partial per block there for the next window.
// ---------------------------------------------------------------------------
//
// FOLD (round 6, the row_fix fold): the previous window's
// leaving rows are rewritten by this launch instead of a row_fix launch after
// its flush.  `pw` is that window's buffer set; if it owes its fix (pw.fix: G
// set by its chain, no gated row_fix since), every thread first rewrites the
// previous window's last-leaving rows r_L of ITS OWN column j when j took the
// flush's fast path there (tag == that window's epoch, no flags): p_L[j], then
// the later slots' msub with f_s[r_L] -- row_fix's arithmetic, from pw.Pf (the
// p history, slot-major) and pw.frt (f_s[r_L]), both stored by that chain as
// side stores of its slots.  The stores are write-through and drained before the
// block's start-handshake arrival, so after the handshake every block reads
// them: the norm phase gathers row r_q on the columns its thread rewrote
// itself, and the ratio phase reads a rewritten row with coherent (sc1) loads.
// This launch then owes its own fix (G[win.sid] = its epoch); the next fold
// chain or a gated row_fix settles it.
// ---------------------------------------------------------------------------
template <int KMAX, int CB, bool FOLD = false>
__global__ __launch_bounds__(CB) void chain_kernel(
    Key* __restrict__ enter_part, State* st, const Params* __restrict__ prm, int n_ep,
    const double* __restrict__ A, int64_t ld, int64_t m, int64_t N, double* __restrict__ obj,
    Window win, int npiv, int64_t* __restrict__ basis, int64_t* __restrict__ hist,
    unsigned long long* gr_enter_, unsigned long long* gr_ratio_, int cpb, int rpb,
    const ChainPeers* __restrict__ /*pe: shards only*/, Window pw = Window{}, int nfix = 0,
    double* Aw = nullptr) {
  static_assert(KMAX <= 32, "slots are lane-indexed and fit the window buffers");
  constexpr int NW = CB / 64;
  static_assert(!FOLD || KMAX * CB * 16 <= 128 * 1024, "the fold reads the LDS f histories");
  // LEAN (round 5; wherever the LDS histories allow it):
  // the slot chains carry no per-slot "s < q" select.  A slot s >= q is an exact identity instead: its f and p
  // histories are +0 (LDS zeroed at the window start, record lanes >= q are
  // +0), and v - (+0 * +0) = v for every v, -0 and NaN included.  Only a
  // chunk of CH slots is guarded, by a uniform branch.  (Round 5 also tried
  // the norm phase's zero-p slots on that chain, p taken as +0: slower, 8.77
  // against 8.52 us per pivot, profiles/r05/ab_chain_lean.jsonl.)
  // LH: the window histories f_s[i] (rows) and p_s[j] (columns) live in LDS,
  // slot-major, one column per thread: a phase reads its thread's slots once
  // and appends one, instead of a 2*KMAX-select register update on the path
  // to the record (and the winner's history is published straight from them)
  constexpr bool LH = KMAX * CB * 16 <= 128 * 1024;
  constexpr bool LEAN = LH && KMAX % 4 == 0;
  constexpr int CH = LEAN ? 4 : KMAX % 8 == 0 ? 8 : KMAX % 4 == 0 ? 4 : 2;
  __shared__ double fsl[LH ? KMAX : 1][LH ? CB : 1];
  __shared__ double psl[LH ? KMAX : 1][LH ? CB : 1];
  __shared__ double hl33[NW];  // LH: the wave winners' RHS (the ratio record's extra)
  // one block per CU: the record protocol is validated for that residency
  // (with LH the histories already take most of it)
  constexpr int PIN = LH ? (82 * 1024 - KMAX * CB * 16 > 8 ? (82 * 1024 - KMAX * CB * 16) / 8 : 1)
                         : 80 * 128;
  __shared__ double lds_pin[PIN];
  __shared__ int64_t bc_idx;  // the winner handed from wave 0 to the block
  __shared__ double bc_val;
  __shared__ int bc_blk;
  __shared__ KeyP sk[NW];       // the waves' best keys (payload b = wave index)
  __shared__ double hl[LH ? 1 : NW][34];  // their winners' histories (+ [33]: the row's RHS)
  gu64* gr_enter = (gu64*)gr_enter_;
  gu64* gr_ratio = (gu64*)gr_ratio_;
  const int B = gridDim.x;
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = t >> 6;
  const bool w0 = t < 64;
  const bool leader = b == 0 && t == 0;
  SPX_PROBE(KMAX + 2, 0, 0, true);  // (probe build: the chain's entry)
  // FOLD: does the previous window's set owe its fix (G set, no gated row_fix
  // since)?  Nothing writes pw.fix during this launch.
  int32_t fg = 0;
  bool pend = false;
  if constexpr (FOLD) {
    fg = pw.fix[pw.sid];
    pend = fg != 0 && fg != pw.fix[2 + pw.sid];
  }
  // --- everything that does not depend on a pivot, in one batch ---
  const int32_t status0 = st->status;
  const int64_t forced_c = st->forced_c;
  const int64_t forced_r = st->forced_r;
  const int64_t it0 = st->iters;
  const int64_t hist_cap = st->hist_cap;
  const int64_t hs_bound = st->hs_ticks;
  const uint32_t E = *win.epoch;
  const int32_t rule = prm->rule;
  const double eps_piv = prm->eps_piv;
  const double eps_opt = prm->eps_opt;
  const int64_t n_enter = prm->n_enter;
  const int64_t iter_limit = prm->iter_limit;
  const bool skip = prm->skip_zero != 0;
  const uint32_t W = (E + 1u) & TAG_EPOCH;  // this window's epoch
  // my column and my row
  const int64_t j = (int64_t)b * cpb + t;
  const bool jlive = t < cpb && j < N;
  const int64_t jc = jlive ? j : 0;
  // rows sit on waves 1.. when they fit (roff = 64), so the polling wave 0
  // issues no row-side stores (f_q) that its next poll's vmcnt wait would
  // also have to drain; the pivot bookkeeping is stored by the last thread
  const int roff = rpb <= CB - 64 ? 64 : 0;
  const int64_t i = (int64_t)b * rpb + (t - roff);
  const bool ilive = t >= roff && t - roff < rpb && i < m;
  const int64_t ic = ilive ? i : 0;
  double o = obj[jc];
  uint32_t tg = jlive ? win.tag[jc] : 0u;
  const uint32_t tg0 = tg;
  // The RHS column N-1 is never an entering candidate and its pivot-row value
  // is the ratio record's p_q[rhs] (the row owner's current RHS / pivot), so
  // when the host sizes the grid by the N-1 candidate columns (B * cpb == N-1:
  // 64 blocks at config 3, a single-pass poll) the last thread of the last
  // block keeps it beside its own column: objective value, tag, p history.
  const bool xown = (int64_t)B * cpb == N - 1 && b == B - 1 && t == CB - 1;
  double ox = xown ? obj[N - 1] : 0.0;
  uint32_t tgx = xown ? win.tag[N - 1] : 0u;
  const uint32_t tgx0 = tgx;
  uint32_t zmx = 0u;
  __shared__ double pxl[KMAX];  // p_s[N-1] (xown only)
  double bcur = A[(N - 1) * ld + ic];   // current RHS of my row (stale + applied slots)
  int64_t bas = basis[ic];              // basis[i] (Bland's tie key)
  double fs[KMAX], ps[KMAX];            // f_s[i], p_s[j] of this window
#pragma unroll
  for (int s = 0; s < KMAX; ++s) fs[s] = ps[s] = 0.0;
  int64_t slot_r = 0, slot_c = -1;      // lane s: (r_s, c_s)
  // per-thread slot masks (bit s): my row left at slot s (i == r_s), my column
  // entered at slot s (j == c_s), p_s[j] == 0 under the skip rule
  uint32_t rmask = 0u, cmask = 0u, zmask = 0u;
  // FOLD: the previous window's leaving rows (lane s: r_s and whether s is
  // the row's last leaving slot; xfr[L][s] = f_s[r_L] from pw.frt, in LDS)
  // and my column's p history there (pw.Pf, slot-major) -- loaded with the
  // kernel's first batch, whether or not a fix is owed (one round trip)
  __shared__ double xfr[FOLD ? KMAX : 1][FOLD ? KMAX : 1];
  int64_t xr = -1;
  int xl = 0, xmk = 0;
  if constexpr (FOLD) {
    constexpr int PERT = (KMAX * KMAX + CB - 1) / CB;
    double fv[PERT];
#pragma unroll
    for (int u = 0; u < PERT; ++u) {
      const int x = t + CB * u;
      fv[u] = x < KMAX * KMAX ? pw.frt[(x / KMAX) * KW + x % KMAX] : 0.0;
    }
    xr = lane < KMAX ? pw.r[lane] : -1;
    const int pm = lane < KMAX ? pw.made[lane] : 0;
    double pp[KMAX];
#pragma unroll
    for (int s2 = 0; s2 < KMAX; ++s2) pp[s2] = pw.Pf[(int64_t)s2 * N + jc];
    // the RHS column's p history by lane (the wave of the last thread, when
    // it keeps the RHS column beside its own: xown)
    const bool xw = (int64_t)B * cpb == N - 1 && b == B - 1 && w == NW - 1;
    const double prl = xw && lane < KMAX ? pw.Pf[(int64_t)lane * N + N - 1] : 0.0;
    if (pend) {
      const uint32_t fe = (uint32_t)fg & TAG_EPOCH;  // that window's epoch
      const bool pfj = jlive && tg0 == fe;  // my column took its fast path there
      xmk = __popcll(__ballot(pm != 0));  // (a prefix: its chain cleared the rest)
      bool last = lane < xmk;
#pragma unroll
      for (int s2 = 1; s2 < KMAX; ++s2)
        last &= !(s2 > lane && s2 < xmk && rdlane64(xr, s2) == xr);
      xl = last ? 1 : 0;
#pragma unroll
      for (int u = 0; u < PERT; ++u) {
        const int x = t + CB * u;
        if (x < KMAX * KMAX) xfr[x / KMAX][x % KMAX] = fv[u];
      }
      __syncthreads();
      // row_fix's value of (r_L, j) for each last-leaving slot L, stored
      // write-through (wave-uniform L: one msub chain per lane)
#pragma unroll
      for (int L = 0; L < KMAX; ++L) {
        if (!__builtin_amdgcn_readlane(xl, L)) continue;
        const int64_t rL = rdlane64(xr, L);
        double x = pp[L];
#pragma unroll
        for (int s2 = L + 1; s2 < KMAX; ++s2)
          if (s2 < xmk) x = msub(x, xfr[L][s2], pp[s2]);
        if (pfj) wt_store(const_cast<double*>(A) + jc * ld + rL, x);
      }
      // the RHS column (xown): its wave's lane L takes slot L
      if (xw && (uint32_t)__builtin_amdgcn_readlane((int)tgx0, 63) == fe) {
        const int L = lane < KMAX ? lane : 0;
        double x = prl;
#pragma unroll
        for (int s2 = 1; s2 < KMAX; ++s2) {
          const double p_s = rdlane(prl, s2);
          if (s2 > L && s2 < xmk) x = msub(x, xfr[L][s2], p_s);
        }
        if (xl) wt_store(const_cast<double*>(A) + (N - 1) * ld + xr, x);
      }
      drain_stores();
      __syncthreads();  // (every store of the block drained before its arrival)
      SPX_PROBE(KMAX + 2, 0, 1, true);  // (probe build: the fold's rows stored)
    }
  }
  if (t == 0) lds_pin[b % PIN] = 0.0;
  SPX_PROBE_CHAIN_HW();
  if constexpr (LEAN) {  // slots s >= q read +0 histories (written at slot s only)
#pragma unroll
    for (int s = 0; s < KMAX; ++s) fsl[s][t] = psl[s][t] = 0.0;
  }
  if (status0 != ST_RUNNING) {          // grid-uniform: no pivot in this window
    if (leader) {
      // (the flush counts made slots; a fold set's made slots are exactly its pivots)
      for (int s = 0; s < (FOLD ? KMAX : npiv); ++s) win.made[s] = 0;
      if constexpr (FOLD) win.fix[win.sid] = 0;  // this window owes nothing
    }
    return;
  }
  {
    // start handshake: every block resident, or nothing of this window runs
    gu64* hs = gr_ratio + (size_t)HS_PLANE_1GPU * CHAIN_MAX_BLOCKS;
    const uint64_t t_hs = __builtin_amdgcn_s_memrealtime();
    __shared__ int hs_res;
    if (t == 0) g_store(hs + b, rec_tag(W, 0, GK_START), 0u);
    if (w0) {
      const int res = chain_start<false>(hs, B, B, 1u, hs + CHAIN_MAX_BLOCKS, W, hs_bound, t_hs,
                                         nullptr, st);
      if (t == 0) hs_res = res;
    }
    __syncthreads();
    if (hs_res != 0) {  // (2: ST_FAULT is stored already)
      if (leader) {
        if (hs_res == 1) st->status = ST_NOTRES;
        for (int s = 0; s < (FOLD ? KMAX : npiv); ++s) win.made[s] = 0;
        if constexpr (FOLD) win.fix[win.sid] = 0;
      }
      return;
    }
  }
  SPX_PROBE(KMAX + 2, 0, 2, true);  // (probe build: the handshake passed)
  // FOLD: does my row hold a rewritten value (it left the previous window)?
  // Then column reads of it are coherent (sc1) loads: another block rewrote it
  bool dirty = false, wdirty = false;
  if constexpr (FOLD) {
    if (pend) {
#pragma unroll
      for (int s2 = 0; s2 < KMAX; ++s2)
        dirty |= __builtin_amdgcn_readlane(xl, s2) && rdlane64(xr, s2) == i;
      dirty = dirty && ilive;
      wdirty = __ballot(dirty) != 0ull;
      if (wdirty && dirty) bcur = wt_load(A + (N - 1) * ld + ic);
    }
  }
  if (leader) {
    // the flush's record counter; reset write-through and drained before this
    // block's first record (every other block adds to it only after polling
    // that record)
    __hip_atomic_store((gu32*)win.nlist, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  int q = 0;
  int64_t r_prev = -1;
  double f_prev = 0.0, prhs = 0.0;  // my f_{q-1}[i]; p_{q-1}[rhs] = RHS of r_{q-1} / pivot
  int32_t stop_status = ST_RUNNING;
  for (; q < npiv; ++q) {
    // ================= ratio phase q =================
    SPX_PROBE(q, 0, 0, true);
    int64_t c;
    double zc;
    int wb = 0;
    if (q == 0) {
      // entering partials of the previous kernel (visible: kernel boundary)
      Keys8 kk;
      keys_issue(kk, enter_part, n_ep);
      KeyR e = keys_reduce(kk, enter_part, n_ep);
      wave_min_dpp(e);
      c = e.row;
      zc = c >= 0 ? obj[c] : 0.0;
    } else {
      if (w0) {
        KeyP e;
        const bool ok =
            poll_records<false, 3>(gr_enter, B, rec_tag(W, q - 1, GK_ENTER), rule, e, st);
        if (t == 0) {
          bc_idx = ok ? e.row : -2;
          bc_val = e.a;
          bc_blk = (int)e.b;
        }
        SPX_PROBE_CHAIN(q - 1, 3);
      }
      __syncthreads();
      c = bc_idx;
      zc = bc_val;
      wb = bc_blk;
      if (c == -2) return;  // a wait timed out (ST_FAULT stored)
    }
    SPX_PROBE(q, 0, 1, true);
    if (forced_c >= 0) {
      c = forced_c;
      zc = obj[c];  // (forced pivots are single-pivot windows: q == 0)
    }
    const int64_t it = it0 + q;
    if (c < 0) stop_status = ST_OPTIMAL;
    else if (forced_r < 0 && it >= iter_limit) stop_status = ST_LIMIT;
    if (stop_status != ST_RUNNING) break;  // grid-uniform
    // column c on my row: stale + pending slots, in slot order; p_s[c] (lane
    // s) from the winning entering record's history
    double fv = A[c * ld + ic];
    if constexpr (FOLD) {  // (a row another block rewrote at the window start)
      if (wdirty && dirty) fv = wt_load(A + c * ld + ic);
    }
    if constexpr (LH) {  // my row's f history, read while the gathers are in flight
#pragma unroll
      for (int s = 0; s < KMAX; ++s) fs[s] = fsl[s][t];
    }
    double pcl = 0.0, unused[2];
    if (q > 0 &&
        !load_extras<0>(gr_enter, wb, ENTER_HDR, q, 0, rec_tag(W, q - 1, GK_ENTER), pcl, unused,
                        st))
      return;
    SPX_PROBE(q, 2, 0, fv != 12345.678 && pcl != 12345.678);  // loads arrived
    SPX_PROBE_CHAIN_T(q, 4, fv != 12345.678 && pcl != 12345.678);
    // RHS: apply slot q-1 (the slots before it are already in bcur)
    if (q > 0) bcur = apply_sel(bcur, i == r_prev, false, true, f_prev, prhs, skip);
    // apply_sel's special cases as masks: column c entered earlier in this
    // window or p_s[c] == 0 under the skip rule (uniform: the exact loop), my
    // row left at slot s (rmask: p_s[c] replaces the msub on that lane).
    // Otherwise a slot is one msub (~5 VALU ops instead of ~25).
    fv = ratio_slots<KMAX, CH, LEAN>(fv, fs, pcl, rmask, q, i, c, slot_r, slot_c, skip);
    SPX_PROBE(q, 2, 1, fv != 12345.678);  // slots applied
    SPX_PROBE_CHAIN_T(q, 6, fv != 12345.678);
    if constexpr (LH) {
      fsl[q][t] = fv;
    } else {
#pragma unroll
      for (int s = 0; s < KMAX; ++s) fs[s] = (s == q) ? fv : fs[s];
    }
    f_prev = fv;
    KeyP k = keyp_none();
    if (ilive) {
      if (forced_r >= 0) {
        if (i == forced_r) kmin2(k, 0.0, 0, i, 0.0, 0.0);
      } else if (fv > eps_piv) {
        const double rq = bcur / fv;
        if (rq == rq) kmin2(k, rq, rule == RULE_BLAND ? bas : i, i, 0.0, 0.0);
      }
    }
    SPX_PROBE(q, 0, 2, fv != 12345.678);
    // publish: the wave winner puts its f history and RHS in LDS, the block's
    // winner is published by wave 0 (rows grow with the lane: Dantzig's tie key)
    k = key_of_lane(k, wave_argmin(k.v, k.t, k.row >= 0, rule != RULE_BLAND));
    if (ilive && k.row == i) {
      if constexpr (LH) {
        hl33[w] = bcur;
      } else {
#pragma unroll
        for (int s = 0; s < KMAX; ++s)
          if (s <= q) hl[w][s] = fs[s];
        hl[w][33] = bcur;
      }
    }
    if (lane == 0) sk[w] = KeyP{k.v, k.t, k.row, 0.0, (double)w};
    SPX_PROBE(q, 2, 2, k.v != 12345.678);  // wave argmin + LDS hand-off issued
    __syncthreads();
    SPX_PROBE(q, 2, 3, true);              // every wave of the block arrived
    if (w0) {
      publish_local<NW, true>(gr_ratio, b, rec_tag(W, q, GK_RATIO), q + 1, sk,
                               [&](int ww, int64_t row, int x) -> double {
                                 if constexpr (LH)
                                   return x == 33 ? hl33[ww]
                                                  : fsl[x][(int)(row - (int64_t)b * rpb) + roff];
                                 else
                                   return hl[ww][x];
                               }, q, rule != RULE_BLAND);
      SPX_PROBE_CHAIN(q, 0);
    }
    // f_q for the flush / row_fix (later kernels): stored after the record, so
    // these stores never queue in front of it
    if (ilive) win.F[(int64_t)q * ld + i] = fv;
    if constexpr (FOLD) {
      // my row left earlier in this window (last at slot L): f_q of it, for
      // the next fold chain's rewrite of the row (win.frt[L][q])
      if (ilive && rmask != 0u) win.frt[(31 - __builtin_clz(rmask)) * KW + q] = fv;
    }
    SPX_PROBE(q, 0, 3, true);
    // ================= norm phase q =================
    SPX_PROBE(q, 1, 0, true);
    if (w0) {
      KeyP rk;
      const unsigned rtag = rec_tag(W, q, GK_RATIO);
      const bool ok = rule == RULE_BLAND
                          ? poll_records<true, 4>(gr_ratio, B, rtag, rule, rk, st)
                          : poll_records<true, 3>(gr_ratio, B, rtag, rule, rk, st);
      if (t == 0) {
        bc_idx = ok ? rk.row : -2;
        bc_blk = (int)rk.b;
      }
      SPX_PROBE_CHAIN(q, 1);
    }
    __syncthreads();
    const int64_t r = bc_idx;
    wb = bc_blk;
    if (r == -2) return;
    SPX_PROBE(q, 1, 1, true);
    if (q == 0 && leader) *win.epoch = W;  // every block has read E (its record carries W)
    if (r < 0) {
      stop_status = ST_UNBOUNDED;
      break;
    }
    // row r on my column: stale + pending slots.  f_s[r] (lane s <= q, lane q
    // the pivot element) and the row's RHS from the winning ratio record
    double v = A[jc * ld + r];
    if constexpr (LH) {  // my column's p history, read while the gathers are in flight
#pragma unroll
      for (int s = 0; s < KMAX; ++s) ps[s] = psl[s][t];
    }
    double frl = 0.0, ex[2];
    if (!load_extras<1>(gr_ratio, wb, RATIO_HDR + 2, q + 1, RATIO_HDR, rec_tag(W, q, GK_RATIO),
                        frl, ex, st))
      return;
    SPX_PROBE(q, 3, 0, v != 12345.678 && frl != 12345.678);  // loads arrived
    SPX_PROBE_CHAIN_T(q, 5, v != 12345.678 && frl != 12345.678);
    const double piv = rdlane(frl, q);
    prhs = ex[0] / piv;  // p_q[rhs]: lazy_norm's p = v / piv of the RHS column
    // Special cases as masks: row r left earlier in the window (uniform: the
    // exact loop), my column entered at slot s (cmask: the value becomes 0),
    // p_s[j] == 0 under the skip rule (zmask: the value is kept)
    const uint32_t qmn = (1u << q) - 1u;
    const bool zb = (zmask & qmn) != 0u;
    // LEAN: lane q holds the pivot element, which slot q of a chunk must not
    // see (piv * +0 may be -0); lanes > q are +0 already
    v = norm_slots<KMAX, CH, LEAN>(v, ps, frl, zmask, cmask, q, jlive, r, jc, slot_r, slot_c, skip);
    SPX_PROBE(q, 3, 1, v != 12345.678);  // slots applied
    SPX_PROBE_CHAIN_T(q, 7, v != 12345.678);
    KeyP ek;
    double pq;  // p_q[j]
    norm_update<KMAX, LH>(ek, pq, ps, zmask, cmask, o, tg, jlive, j, c, q, v, piv, zc, skip, zb, W,
                          n_enter, eps_opt, rule, xown, zmx, ox, tgx, prhs, qmn, pxl);
    if (ilive && i == r) bas = c;
    rmask |= (i == r) ? (1u << q) : 0u;
    if (lane == q) {
      slot_r = r;
      slot_c = c;
    }
    r_prev = r;
    SPX_PROBE(q, 1, 2, v != 12345.678);
    ek = key_of_lane(ek, wave_argmin(ek.v, ek.t, ek.row >= 0, true));  // columns grow with the lane
    if constexpr (LH) {
      psl[q][t] = pq;
    } else if (q + 1 < npiv && jlive && ek.row == j) {
#pragma unroll
      for (int s = 0; s < KMAX; ++s)
        if (s <= q) hl[w][s] = ps[s];
    }
    if (lane == 0) sk[w] = KeyP{ek.v, ek.t, ek.row, ek.a, (double)w};
    SPX_PROBE(q, 3, 2, ek.v != 12345.678);  // wave argmin + LDS hand-off issued
    __syncthreads();
    SPX_PROBE(q, 3, 3, true);               // every wave of the block arrived
    if (w0) {
      if (q + 1 < npiv) {
        publish_local<NW, false>(gr_enter, b, rec_tag(W, q, GK_ENTER), q + 1, sk,
                                  [&](int ww, int64_t col, int x) -> double {
                                    if constexpr (LH)
                                      return psl[x][(int)(col - (int64_t)b * cpb)];
                                    else
                                      return hl[ww][x];
                                  }, q, true);
      } else if (t == 0) {
        // the next window's pivot-0 partial (read after the kernel boundary)
        KeyP kb = sk[0];
#pragma unroll
        for (int x = 1; x < NW; ++x) kmin2(kb, sk[x].v, sk[x].t, sk[x].row, sk[x].a, sk[x].b);
        store_key(enter_part + b, KeyR{kb.v, kb.t, kb.row});
        // the next window reduces n_ep partials (norm<INIT>'s per-WG count can
        // exceed B, e.g. 512-thread blocks): the ones past this grid's must not
        // keep an earlier kernel's keys
        for (int x = b + B; x < n_ep; x += B) store_key(enter_part + x, keyr_none());
      }
      SPX_PROBE_CHAIN(q, 2);
    }
    // stores for later kernels, after the record (never queued in front of it):
    if constexpr (FOLD) {
      // p_q by column, slot-major (win.Pf), for the next fold chain; the
      // polling wave's columns are stored by the last wave (from LDS: psl is
      // complete after the barrier above), so the poller issues no stores
      if (w > 0 && jlive) win.Pf[(int64_t)q * N + j] = pq;
      if (w == NW - 1) {
        const int64_t j0 = (int64_t)b * cpb + lane;
        if (lane < cpb && j0 < N) win.Pf[(int64_t)q * N + j0] = psl[q][lane];
      }
      if (xown) win.Pf[(int64_t)q * N + N - 1] = prhs;
    }
    // the pivot's bookkeeping (the flush and row_fix read p from the records)
    if (b == 0 && t == CB - 1) {  // block 0's last thread: not in the polling wave
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

    SPX_PROBE(q, 1, 3, true);
  }
  // ---- the window ends after slot q (q pivots made) ----
  if (stop_status != ST_RUNNING && leader) {
    st->status = stop_status;
    if (stop_status == ST_OPTIMAL) st->c_next = -1;
    for (int s = q; s < npiv; ++s) win.made[s] = 0;
  }
  if constexpr (FOLD) {
    if (leader) {
      // a fold set's made slots are exactly its pivots (the next fold chain
      // counts them), and it owes its leaving rows' fix: G = its epoch
      // (bit 30 set, never 0)
      for (int s = q; s < KMAX; ++s) win.made[s] = 0;
      win.fix[win.sid] = q > 0 ? (int32_t)(W | 0x40000000u) : 0;
    }
  }
  if (jlive) {
    obj[j] = o;
    if (tg != tg0) win.tag[j] = tg;
  }
  if (xown) {
    obj[N - 1] = ox;
    if (tgx != tgx0) win.tag[N - 1] = tgx;
  }
  if (q == 0) return;  // no pivot made: nothing to compact (the flush sees nm == 0)
  // compact the window's touched columns into records for the flush (as
  // lazy_norm's last slot): wave ballot + LDS prefix + one atomic per block;
  // the RHS column (xown) follows its wave's own columns
  __shared__ int wcnt[NW];
  __shared__ int base;
  compact_records<KMAX, NW>(win, N, q, W, jlive, xown, j, tg, tgx, pxl, t, lane, w, wcnt, base,
                            [&](int s) -> double {
                              if constexpr (LH) return psl[s][t];
                              else return ps[s];
                            });
}

// ---------------------------------------------------------------------------
// chain_shard_kernel<KMAX, CB>: chain_kernel for this rank's row block of a
// row-sharded tableau.  The columns, objective row and entering
// exchange are replicated per rank (every rank computes the same values), the
// ratio exchange is global (every block's record goes to every rank's buffer,
// polled locally), and the leaving row's stale values are gathered from the
// owner's tableau through a peer pointer.  Rows are local (i), records, slots
// and the basis speak global rows (ig = row0 + i).  pe: the peers' table, in
// device memory (a by-value kernel argument of its size measurably slowed the
// chain).  The single-GPU chain_kernel is this kernel with one rank, kept as
// its own body: folded into this one it measured ~1 us per pivot slower
// (register allocation of a 254-VGPR kernel; profiles/r03/ab_chain_*.jsonl).
// ---------------------------------------------------------------------------
template <int KMAX, int CB>
__global__ __launch_bounds__(CB) void chain_shard_kernel(
    Key* __restrict__ enter_part, State* st, const Params* __restrict__ prm, int n_ep,
    const double* __restrict__ A, int64_t ld, int64_t m, int64_t N, double* __restrict__ obj,
    Window win, int npiv, int64_t* __restrict__ basis, int64_t* __restrict__ hist,
    unsigned long long* gr_enter_, unsigned long long* gr_ratio_, int cpb, int rpb,
    const ChainPeers* __restrict__ pe, Window /*pw: chain_kernel's fold only*/, int /*nfix*/,
    double* /*Aw*/) {
  static_assert(KMAX <= 32, "slots are lane-indexed and fit the window buffers");
  constexpr int NW = CB / 64;

  // LH: the window histories f_s[i] (rows) and p_s[j] (columns) live in LDS,
  // slot-major, one column per thread: a phase reads its thread's slots once
  // and appends one, instead of a 2*KMAX-select register update on the path
  // to the record (and the winner's history is published straight from them)
  constexpr bool LH = KMAX * CB * 16 <= 128 * 1024;
  // LEAN: chain_kernel's guard-free slot chains (slots s >= q are identities
  // on +0 histories; only chunks of CH slots are guarded)
  constexpr bool LEAN = LH && KMAX % 4 == 0;
  constexpr int CH = LEAN ? 4 : KMAX % 8 == 0 ? 8 : KMAX % 4 == 0 ? 4 : 2;
  __shared__ double fsl[LH ? KMAX : 1][LH ? CB : 1];
  __shared__ double psl[LH ? KMAX : 1][LH ? CB : 1];
  __shared__ double hl33[NW];  // LH: the wave winners' RHS (the ratio record's extra)
  // one block per CU: the record protocol is validated for that residency
  // (with LH the histories already take most of it)
  constexpr int PIN = LH ? (82 * 1024 - KMAX * CB * 16 > 8 ? (82 * 1024 - KMAX * CB * 16) / 8 : 1)
                         : 80 * 128;
  __shared__ double lds_pin[PIN];
  __shared__ int64_t bc_idx;  // the winner handed from wave 0 to the block
  __shared__ double bc_val;
  __shared__ int bc_blk;
  __shared__ KeyP sk[NW];       // the waves' best keys (payload b = wave index)
  __shared__ double hl[LH ? 1 : NW][34];  // their winners' histories (+ [33]: the row's RHS)
  gu64* gr_enter = (gu64*)gr_enter_;
  gu64* gr_ratio = (gu64*)gr_ratio_;
  const int B = gridDim.x;
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = t >> 6;
  const bool w0 = t < 64;
  const bool leader = b == 0 && t == 0;
  // --- everything that does not depend on a pivot, in one batch ---
  const int32_t status0 = st->status;
  const int64_t forced_c = st->forced_c;
  const int64_t forced_r = st->forced_r;
  const int64_t it0 = st->iters;
  const int64_t hist_cap = st->hist_cap;
  const int64_t hs_bound = st->hs_ticks;
  const uint32_t E = *win.epoch;
  const int32_t rule = prm->rule;
  const double eps_piv = prm->eps_piv;
  const double eps_opt = prm->eps_opt;
  const int64_t n_enter = prm->n_enter;
  const int64_t iter_limit = prm->iter_limit;
  const bool skip = prm->skip_zero != 0;
  const uint32_t W = (E + 1u) & TAG_EPOCH;  // this window's epoch (the same on every rank)
  // my rank's rows start at row0; the ratio records of all nr * B blocks are
  // polled (block slot rank * B + b, planes RS apart)
  const int rank = pe->rank;
  const int nr = pe->nranks;
  const int64_t row0 = pe->row0[rank];
  constexpr int RS = CHAIN_SH_SLOTS;
  const int BR = nr * B;
  const int bs = rank * B + b;
  const bool push = pe->push != 0;
  const int64_t NI = inbox_stride(N);
  // rank 0's time-limit stop request rides in its ratio records (bit 31 of
  // granule 3); read once per window, so every rank stops at the window's start
  const unsigned stopbit =
      (rank == 0 && pe->stop_req &&
       __hip_atomic_load(const_cast<int32_t*>(pe->stop_req), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM) != 0)
          ? 1u : 0u;
  // the ratio buffer of pivot it0 + q: two halves by pivot parity (a rank's
  // entering exchange is local, so it may publish ratio q + 1 before a peer
  // has read ratio q; never q + 2)
  auto ratio_buf = [&](int d, int qq) -> gu64* {
    return (gu64*)pe->ratio[d] + (size_t)((it0 + qq) & 1) * RATIO_REC * RS;
  };
  // rank d's inbox half for pivot it0 + qq (owner-push): low words, then high
  auto inbox = [&](int d, int qq) -> gu64* {
    return (gu64*)pe->ratio[d] + (size_t)INBOX_PLANE_SHARD * RS + (size_t)((it0 + qq) & 1) * 2 * NI;
  };
  (void)gr_ratio;
  // my column and my row
  const int64_t j = (int64_t)b * cpb + t;
  const bool jlive = t < cpb && j < N;
  const int64_t jc = jlive ? j : 0;
  // rows sit on waves 1.. when they fit (roff = 64), so the polling wave 0
  // issues no row-side stores (f_q) that its next poll's vmcnt wait would
  // also have to drain; the pivot bookkeeping is stored by the last thread
  const int roff = rpb <= CB - 64 ? 64 : 0;
  const int64_t i = (int64_t)b * rpb + (t - roff);  // local row
  const bool ilive = t >= roff && t - roff < rpb && i < m;
  const int64_t ic = ilive ? i : 0;
  const int64_t ig = row0 + i;  // global row (what records, slots and basis speak)
  double o = obj[jc];
  uint32_t tg = jlive ? win.tag[jc] : 0u;
  const uint32_t tg0 = tg;
  // The RHS column N-1 is never an entering candidate and its pivot-row value
  // is the ratio record's p_q[rhs] (the row owner's current RHS / pivot), so
  // when the host sizes the grid by the N-1 candidate columns (B * cpb == N-1:
  // 64 blocks at config 3, a single-pass poll) the last thread of the last
  // block keeps it beside its own column: objective value, tag, p history.
  const bool xown = (int64_t)B * cpb == N - 1 && b == B - 1 && t == CB - 1;
  double ox = xown ? obj[N - 1] : 0.0;
  uint32_t tgx = xown ? win.tag[N - 1] : 0u;
  const uint32_t tgx0 = tgx;
  uint32_t zmx = 0u;
  __shared__ double pxl[KMAX];  // p_s[N-1] (xown only)
  double bcur = A[(N - 1) * ld + ic];   // current RHS of my row (stale + applied slots)
  int64_t bas = basis[row0 + ic];       // basis[ig] (Bland's tie key)
  double fs[KMAX], ps[KMAX];            // f_s[i], p_s[j] of this window
#pragma unroll
  for (int s = 0; s < KMAX; ++s) fs[s] = ps[s] = 0.0;
  int64_t slot_r = 0, slot_c = -1;      // lane s: (r_s, c_s)
  // per-thread slot masks (bit s): my row left at slot s (i == r_s), my column
  // entered at slot s (j == c_s), p_s[j] == 0 under the skip rule
  uint32_t rmask = 0u, cmask = 0u, zmask = 0u;
  if (t == 0) lds_pin[b % PIN] = 0.0;
  if constexpr (LEAN) {  // slots s >= q read +0 histories (written at slot s only)
#pragma unroll
    for (int s = 0; s < KMAX; ++s) fsl[s][t] = psl[s][t] = 0.0;
  }
  if (status0 != ST_RUNNING) {          // grid-uniform: no pivot in this window
    if (leader)
      for (int s = 0; s < npiv; ++s) win.made[s] = 0;  // (the flush counts made slots)
    return;
  }
  {
    // start handshake over this rank's device group (the ranks sharing its
    // GPU), then every group's verdict: every block of every rank resident, or
    // nothing of this window runs on any rank
    const int grp = pe->group;
    gu64* hs = (gu64*)pe->ratio[pe->gleader[grp]] + (size_t)HS_PLANE_SHARD * RS;
    const uint64_t t_hs = __builtin_amdgcn_s_memrealtime();
    __shared__ int hs_res;
    if (t == 0) g_store<true>(hs + bs, rec_tag(W, 0, GK_START), 0u);
    if (w0) {
      const int res = chain_start<true>(hs, BR, B, pe->gmask[grp], hs + RS, W, hs_bound, t_hs,
                                        pe, st);
      if (t == 0) hs_res = res;
    }
    __syncthreads();
    if (hs_res != 0) {  // (2: ST_FAULT is stored already)
      if (b == 0 && t == 0) {
        if (hs_res == 1) st->status = ST_NOTRES;
        for (int s = 0; s < npiv; ++s) win.made[s] = 0;
      }
      return;
    }
  }
  if (leader) {
    // the flush's record counter; reset write-through and drained before this
    // block's first record (every other block adds to it only after polling
    // that record)
    __hip_atomic_store((gu32*)win.nlist, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  int q = 0;
  int64_t r_prev = -1;
  double f_prev = 0.0, prhs = 0.0;  // my f_{q-1}[i]; p_{q-1}[rhs] = RHS of r_{q-1} / pivot
  int32_t stop_status = ST_RUNNING;
  for (; q < npiv; ++q) {
    // ================= ratio phase q =================
    SPX_PROBE(q, 0, 0, true);
    int64_t c;
    double zc;
    int wb = 0;
    if (q == 0) {
      // entering partials of the previous kernel (visible: kernel boundary)
      Keys8 kk;
      keys_issue(kk, enter_part, n_ep);
      KeyR e = keys_reduce(kk, enter_part, n_ep);
      wave_min_dpp(e);
      c = e.row;
      zc = c >= 0 ? obj[c] : 0.0;
    } else {
      if (w0) {
        KeyP e;
        const bool ok = poll_records<false, 3>(gr_enter, B,
                                               rec_tag(W, q - 1, GK_ENTER), rule, e, st);
        if (t == 0) {
          bc_idx = ok ? e.row : -2;
          bc_val = e.a;
          bc_blk = (int)e.b;
        }
        SPX_PROBE_CHAIN(q - 1, 3);
      }
      __syncthreads();
      c = bc_idx;
      zc = bc_val;
      wb = bc_blk;
      if (c == -2) return;  // a wait timed out (ST_FAULT stored)
    }
    SPX_PROBE(q, 0, 1, true);
    if (forced_c >= 0) {
      c = forced_c;
      zc = obj[c];  // (forced pivots are single-pivot windows: q == 0)
    }
    const int64_t it = it0 + q;
    if (c < 0) stop_status = ST_OPTIMAL;
    else if (forced_r < 0 && it >= iter_limit) stop_status = ST_LIMIT;
    if (stop_status != ST_RUNNING) break;  // grid-uniform
    // column c on my row: stale + pending slots, in slot order; p_s[c] (lane
    // s) from the winning entering record's history
    double fv = A[c * ld + ic];
    if constexpr (LH) {  // my row's f history, read while the gathers are in flight
#pragma unroll
      for (int s = 0; s < KMAX; ++s) fs[s] = fsl[s][t];
    }
    double pcl = 0.0, unused[2];
    if (q > 0 &&
        !load_extras<0>(gr_enter, wb, ENTER_HDR, q, 0,
                        rec_tag(W, q - 1, GK_ENTER), pcl, unused, st))
      return;
    SPX_PROBE(q, 2, 0, fv != 12345.678 && pcl != 12345.678);  // loads arrived
    // RHS: apply slot q-1 (the slots before it are already in bcur)
    if (q > 0) bcur = apply_sel(bcur, ig == r_prev, false, true, f_prev, prhs, skip);
    // apply_sel's special cases as masks: column c entered earlier in this
    // window or p_s[c] == 0 under the skip rule (uniform: the exact loop), my
    // row left at slot s (rmask: p_s[c] replaces the msub on that lane).
    // Otherwise a slot is one msub (~5 VALU ops instead of ~25).
    fv = ratio_slots<KMAX, CH, LEAN>(fv, fs, pcl, rmask, q, ig, c, slot_r, slot_c, skip);
    SPX_PROBE(q, 2, 1, fv != 12345.678);  // slots applied
    if constexpr (LH) {
      fsl[q][t] = fv;
    } else {
#pragma unroll
      for (int s = 0; s < KMAX; ++s) fs[s] = (s == q) ? fv : fs[s];
    }
    f_prev = fv;
    KeyP k = keyp_none();
    if (ilive) {
      if (forced_r >= 0) {
        if (ig == forced_r) kmin2(k, 0.0, 0, ig, 0.0, 0.0);
      } else if (fv > eps_piv) {
        const double rq = bcur / fv;
        if (rq == rq) kmin2(k, rq, rule == RULE_BLAND ? bas : ig, ig, 0.0, 0.0);
      }
    }
    SPX_PROBE(q, 0, 2, fv != 12345.678);
    // publish: the wave winner puts its f history and RHS in LDS, the block's
    // winner is published by wave 0 (rows grow with the lane: Dantzig's tie key)
    k = key_of_lane(k, wave_argmin(k.v, k.t, k.row >= 0, rule != RULE_BLAND));
    if (ilive && k.row == ig) {
      if constexpr (LH) {
        hl33[w] = bcur;
      } else {
#pragma unroll
        for (int s = 0; s < KMAX; ++s)
          if (s <= q) hl[w][s] = fs[s];
        hl[w][33] = bcur;
      }
    }
    if (lane == 0) sk[w] = KeyP{k.v, k.t, k.row, 0.0, (double)w};
    SPX_PROBE(q, 2, 2, k.v != 12345.678);  // wave argmin + LDS hand-off issued
    __syncthreads();
    SPX_PROBE(q, 2, 3, true);              // every wave of the block arrived
    if (w0) {
      publish_record<NW, true, true, RS>([&](int d) { return ratio_buf(d, q) + bs; }, nr,
                                   rec_tag(W, q, GK_RATIO), q + 1, sk,
                                   [&](int ww, int64_t row, int x) -> double {
                                     if constexpr (LH)
                                       return x == 33 ? hl33[ww]
                                                      : fsl[x][(int)(row - row0 - (int64_t)b * rpb) +
                                                               roff];
                                     else
                                       return hl[ww][x];
                                   },
                                   stopbit, rule != RULE_BLAND);
      SPX_PROBE_CHAIN(q, 0);
    }
    // f_q for the flush / row_fix (later kernels): stored after the record, so
    // these stores never queue in front of it
    if (ilive) win.F[(int64_t)q * ld + i] = fv;
    SPX_PROBE(q, 0, 3, true);
    // ================= norm phase q =================
    SPX_PROBE(q, 1, 0, true);
    if (w0) {
      KeyP rk;
      const unsigned rtag = rec_tag(W, q, GK_RATIO);
      bool stopq = false;
      const bool ok =
          poll_records<true, 4, true, RS>(ratio_buf(rank, q), BR, rtag, rule, rk, st, &stopq);
      if (t == 0) {
        bc_idx = ok ? (stopq ? -3 : rk.row) : -2;
        bc_blk = (int)rk.b;
      }
      SPX_PROBE_CHAIN(q, 1);
    }
    __syncthreads();
    const int64_t r = bc_idx;
    wb = bc_blk;
    if (r == -2) return;
    SPX_PROBE(q, 1, 1, true);
    if (q == 0 && leader) *win.epoch = W;  // every block has read E (its record carries W)
    if (r == -3) {  // rank 0's time-limit stop, seen by every rank at this pivot
      stop_status = ST_LIMIT;
      break;
    }
    if (r < 0) {
      stop_status = ST_UNBOUNDED;
      break;
    }
    // row r on my column: stale + pending slots.  f_s[r] (lane s <= q, lane q
    // the pivot element) and the row's RHS from the winning ratio record
    double v = 0.0;  // the owner's stale row (a peer's tableau unless it is mine)
    const int own = wb / B;
    const unsigned rtag = rec_tag(W, q, GK_RATIO);
    if (own == rank) v = A[jc * ld + (r - row0)];
    else if (!push) v = sys_load(pe->A[own] + jc * pe->ld[own] + (r - pe->row0[own]));
    if constexpr (LH) {  // my column's p history, read while the gathers are in flight
#pragma unroll
      for (int s = 0; s < KMAX; ++s) ps[s] = psl[s][t];
    }
    double frl = 0.0, ex[2];
    if (!load_extras<1, true, RS>(ratio_buf(rank, q), wb, RATIO_HDR + 2, q + 1, RATIO_HDR,
                            rtag, frl, ex, st))
      return;
    if (push) {
      if (own == rank) {
        // owner-push: my stale row values into every peer's inbox (contiguous
        // granules per column block; the data is the flag, no fence)
        if (jlive) {
          const unsigned long long x = (unsigned long long)__double_as_longlong(v);
          for (int d = 0; d < nr; ++d) {
            if (d == rank) continue;
            gu64* ib = inbox(d, q);
            g_store<true>(ib + jc, rtag, (unsigned)x);
            g_store<true>(ib + NI + jc, rtag, (unsigned)(x >> 32));
          }
        }
      } else {
        // the owner's push into my inbox: every lane's two granules tagged
        const gu64* ib = inbox(rank, q);
        for (unsigned spins = 0;;) {
          const unsigned long long lo = g_load<true>(ib + jc), hi = g_load<true>(ib + NI + jc);
          const bool good = !jlive || ((unsigned)(lo >> 32) == rtag && (unsigned)(hi >> 32) == rtag);
          if (__all(good)) {
            v = jlive ? g_decode_d(lo, hi) : 0.0;
            break;
          }
          if (spin_fail(spins, st)) return;
        }
      }
    }
    SPX_PROBE(q, 3, 0, v != 12345.678 && frl != 12345.678);  // loads arrived
    const double piv = rdlane(frl, q);
    prhs = ex[0] / piv;  // p_q[rhs]: lazy_norm's p = v / piv of the RHS column
    // Special cases as masks: row r left earlier in the window (uniform: the
    // exact loop), my column entered at slot s (cmask: the value becomes 0),
    // p_s[j] == 0 under the skip rule (zmask: the value is kept)
    const uint32_t qmn = (1u << q) - 1u;
    const bool zb = (zmask & qmn) != 0u;
    // LEAN: lane q holds the pivot element, which slot q of a chunk must not
    // see (piv * +0 may be -0); lanes > q are +0 already
    v = norm_slots<KMAX, CH, LEAN>(v, ps, frl, zmask, cmask, q, jlive, r, jc, slot_r, slot_c, skip);
    SPX_PROBE(q, 3, 1, v != 12345.678);  // slots applied
    KeyP ek;
    double pq;  // p_q[j]
    norm_update<KMAX, LH>(ek, pq, ps, zmask, cmask, o, tg, jlive, j, c, q, v, piv, zc, skip, zb, W,
                          n_enter, eps_opt, rule, xown, zmx, ox, tgx, prhs, qmn, pxl);
    if (ilive && ig == r) bas = c;
    rmask |= (ig == r) ? (1u << q) : 0u;
    if (lane == q) {
      slot_r = r;
      slot_c = c;
    }
    r_prev = r;
    SPX_PROBE(q, 1, 2, v != 12345.678);
    ek = key_of_lane(ek, wave_argmin(ek.v, ek.t, ek.row >= 0, true));  // columns grow with the lane
    if constexpr (LH) {
      psl[q][t] = pq;
    } else if (q + 1 < npiv && jlive && ek.row == j) {
#pragma unroll
      for (int s = 0; s < KMAX; ++s)
        if (s <= q) hl[w][s] = ps[s];
    }
    if (lane == 0) sk[w] = KeyP{ek.v, ek.t, ek.row, ek.a, (double)w};
    SPX_PROBE(q, 3, 2, ek.v != 12345.678);  // wave argmin + LDS hand-off issued
    __syncthreads();
    SPX_PROBE(q, 3, 3, true);               // every wave of the block arrived
    if (w0) {
      if (q + 1 < npiv) {
        publish_record<NW, false>([&](int) { return gr_enter + b; }, 1,
                                  rec_tag(W, q, GK_ENTER), q + 1, sk,
                                  [&](int ww, int64_t col, int x) -> double {
                                    if constexpr (LH)
                                      return psl[x][(int)(col - (int64_t)b * cpb)];
                                    else
                                      return hl[ww][x];
                                  }, 0u, true);
      } else if (t == 0) {
        // the next window's pivot-0 partial (read after the kernel boundary)
        KeyP kb = sk[0];
#pragma unroll
        for (int x = 1; x < NW; ++x) kmin2(kb, sk[x].v, sk[x].t, sk[x].row, sk[x].a, sk[x].b);
        store_key(enter_part + b, KeyR{kb.v, kb.t, kb.row});
        // the next window reduces n_ep partials (norm<INIT>'s per-WG count can
        // exceed B, e.g. 512-thread blocks): the ones past this grid's must not
        // keep an earlier kernel's keys
        for (int x = b + B; x < n_ep; x += B) store_key(enter_part + x, keyr_none());
      }
      SPX_PROBE_CHAIN(q, 2);
    }
    // stores for later kernels, after the record (never queued in front of it):
    // the pivot's bookkeeping (the flush and row_fix read p from the records)
    if (b == 0 && t == CB - 1) {  // block 0's last thread: not in the polling wave
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
    SPX_PROBE(q, 1, 3, true);
  }
  {
    // Window-end barrier: a rank's next kernels (flush, row_fix) rewrite its
    // rows, so none may start while a peer still gathers one of them.  Every
    // block reports once its last row gather has returned (its values were
    // consumed before the last block barrier above); block 0 of every rank
    // waits for all nr * B reports, so no rank's chain launch completes
    // before every rank is done reading.
    // (owner-push: no rank reads another's rows, so no barrier is needed; the
    // inbox halves by pivot parity keep a rank running a slot ahead safe)
    if (w0 && !push) {
      const unsigned dtag = rec_tag(W, 0, GK_DONE);
      if (lane < nr)
        g_store<true>((gu64*)pe->ratio[lane] + (size_t)2 * RATIO_REC * RS + bs, dtag, 0u);
      if (b == 0) {
        const gu64* dp = (const gu64*)pe->ratio[rank] + (size_t)2 * RATIO_REC * RS;
        for (unsigned spins = 0;;) {
          bool ok = true;
          for (int x = lane; x < BR; x += 64) ok &= (unsigned)(g_load<true>(dp + x) >> 32) == dtag;
          if (__all(ok) || spin_fail(spins, st)) break;
        }
      }
    }
  }
  // ---- the window ends after slot q (q pivots made) ----
  if (stop_status != ST_RUNNING && leader) {
    st->status = stop_status;
    if (stop_status == ST_OPTIMAL) st->c_next = -1;
    for (int s = q; s < npiv; ++s) win.made[s] = 0;
  }
  if (jlive) {
    obj[j] = o;
    if (tg != tg0) win.tag[j] = tg;
  }
  if (xown) {
    obj[N - 1] = ox;
    if (tgx != tgx0) win.tag[N - 1] = tgx;
  }
  if (q == 0) return;  // no pivot made: nothing to compact (the flush sees nm == 0)
  // compact the window's touched columns into records for the flush (as
  // lazy_norm's last slot): wave ballot + LDS prefix + one atomic per block;
  // the RHS column (xown) follows its wave's own columns
  __shared__ int wcnt[NW];
  __shared__ int base;
  compact_records<KMAX, NW>(win, N, q, W, jlive, xown, j, tg, tgx, pxl, t, lane, w, wcnt, base,
                            [&](int s) -> double {
                              if constexpr (LH) return psl[s][t];
                              else return ps[s];
                            });
}

}  // namespace spx
