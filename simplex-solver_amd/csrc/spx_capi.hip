// spx_capi.hip — C-ABI of the MI355X simplex pivot engine (declared in include/spx.h).
//
// Host runtime: one context = one HIP stream + the device-resident tableau,
// pivot vectors, reduction partials and a device State block.  The pivot loop
// never round-trips to the host inside a chunk: each host call primes the
// first pivot (norm<INIT> + prime_kernel), then every pivot is two kernels
// (norm -> elim, the elim also running the next pivot's ratio test), and
// chunks of `chunk` pivots are captured once into a hipGraph and replayed; the
// host only reads the State block (pinned) after each chunk to check for
// termination / limits.
//
// Sharded contexts (spx_create_sharded) split the constraint rows across ranks,
// one process per GPU.  Per pivot they run ONE RCCL all-gather: every rank
// contributes [its best leaving-row key | that row normalised]; every rank then
// takes the lexicographic winner (the leaving-row "allreduce-min", which RCCL
// has no MINLOC op for) and the winner's row as the pivot row (the owner's
// broadcast, without a host-known root).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/spx.h"
#include "spx_kernels.hpp"
#include "spx_delayed.hpp"
#include "spx_chain.hpp"

using namespace spx;

// In-process communicator for "virtual ranks": nranks contexts on one GPU,
// driven by nranks host threads.  Same per-pivot exchange as RCCL (all-gather
// of the leaving-row keys, sum of the pivot-row buffers), implemented with
// stream events + a host barrier, so every sharded kernel path can be tested
// with nranks > 1 on a single-GPU machine.  Not capturable in a hipGraph.
struct LoopGroup {
  int n = 0;
  int refs = 0;
  std::string key;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;
  std::vector<spx_ctx*> members;
  // returns false on timeout (a peer died): the group is then broken for good
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return false;
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; }) ||
        broken) {
      broken = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
};

struct spx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;

  // distribution
  int rank = 0, nranks = 1;
  bool sharded = false;
  ncclComm_t comm = nullptr;
  LoopGroup* loop = nullptr;   // in-process virtual ranks instead of RCCL
  hipEvent_t ev_ready = nullptr, ev_done = nullptr;

  // dims
  int64_t m_global = 0, m_local = 0, row0 = 0, N = 0, ld = 0;
  bool loaded = false;

  // device buffers
  double* A = nullptr;     // ld * N, column-major local rows
  double* obj = nullptr;   // N
  double* F = nullptr;     // 2*ld pivot-column snapshots (by pivot parity)
  double* P = nullptr;     // N    pivot row (normalised)
  int* list = nullptr;     // N    compacted columns
  int64_t* basis = nullptr;// m_global
  int64_t* hist = nullptr; // 2 * hist_cap
  Key* enter_part = nullptr;
  Key* ratio_part = nullptr;
  char* sendbuf = nullptr;   // sharded: this rank's all-gather payload
  char* recvbuf = nullptr;   // sharded: nranks payloads
  int64_t gstride = 0;       // payload stride (bytes)
  Params* prm = nullptr;
  State* st = nullptr;
  State* h_st = nullptr;   // pinned mirror
  State* h_poll = nullptr; // pinned [2]: State copies polled one chunk behind (spx_solve)
  int32_t* h_stop = nullptr;  // pinned, device-visible: rank 0's time-limit stop request
  int32_t* d_stop = nullptr;  // (sharded contexts; spx_kernels.hpp stop_requested)
  hipEvent_t ev_poll[2] = {nullptr, nullptr};
  int64_t hist_cap = 0;

  // launch geometry
  int nbn = 1, nbr = 1, rch = 1, G = 1, R = 8;
  int elim_nt = 0;         // bit 0: non-temporal loads, bit 1: non-temporal stores
  int tune_nt = -1;        // -1: automatic (non-temporal stores on tall shards)
  int elim_ilv = 1;        // interleaved column assignment
  int elim_pipe = 1;       // software-pipelined column pairs (+12% on config 3)
  int elim_xcd = 0;        // XCD-aware block swizzle
  // resident flush blocks per CU, by kernel instance (every template instance has
  // its own register / LDS budget, e.g. the guarded partial-window flush)
  std::map<const void*, int> flush_bpc;
  int flush_map = 0;       // flush block -> (row chunk, column group) map
  int flush_tail = FLUSH_TAIL_DEFAULT;  // % of the records rows moved to the tail (spx_delayed.hpp)
  int last_flush_G = 0;    // column groups of the last flush launch
  int last_flush_rch = 0;  // row chunks of the last flush launch
  int n_cu = 0;
  int ld_pad = -1;         // extra doubles per column (-1: auto, 256 for big shards)
  int tune_R = 0;          // 0: automatic
  int tune_wgs = 0;        // 0: automatic (2048)

  // windowed (delayed) elimination: 0 = off (fused per-pivot elimination)
  int win_k = 0;
  // two sets of per-window buffers, alternating by window (wpar: the set of
  // the next window), so window w's buffers survive window w+1's chain, which
  // resolves w's leaving rows (the row_fix fold).  last_fold:
  // the last enqueued window was a fold window (its set may owe its fix: a
  // gated row_fix settles it before a window that is not one, and at the end
  // of every call).  fold: use fold windows (spx_set_row_fix_fold; the
  // persistent single-GPU chain only).
  Window wins[2]{};
  int wpar = 0;
  bool last_fold = false;
  int fold = 0;  // (off by default: measured no faster)
  // persistent pivot chain of a window (spx_chain.hpp): record buffers and mode
  unsigned long long* gr_enter = nullptr;  // ENTER_REC x CHAIN_MAX_BLOCKS granules
  unsigned long long* gr_ratio = nullptr;  // RATIO_REC x CHAIN_MAX_BLOCKS granules
  size_t A_bytes = 0, gr_bytes = 0;
  int epl_alloc = 0, rpl_alloc = 0;  // entering / ratio partial slots allocated
  // row-transfer staging buffer kept between calls when small (transfer_rows)
  double* stage = nullptr;
  size_t stage_bytes = 0;
  int chain_mode = 0;      // 0: persistent chain when it fits, 1: launch per phase
  int chain_min_blocks = 0;
  // admission of the persistent chain (process-wide block budget per device):
  // blocks this context holds, calls holding them (released by a stream host
  // callback once the call's launches have run), and whether the current call
  // was refused (its windows then run the launch-per-phase chain)
  int adm_blocks = 0;
  int adm_calls = 0;
  int adm_deferred = 0;          // calls whose reservation waits for adm_ev (adm_settle)
  hipEvent_t adm_ev = nullptr;   // recorded behind the last such call's launches
  bool chain_denied = false;
  int64_t chain_calls[2] = {0, 0};  // calls run with the persistent / the lazy chain

  // row-sharded persistent chain: every rank's ratio-record
  // buffer and stale tableau, valid for the loaded tableau (spx_peer_*)
  bool peer_ok = false;
  ChainPeers peers{};
  std::vector<void*> ipc_open;  // IPC-mapped peer buffers (closed on reload / destroy)
  // Exported buffers (round 5).  A buffer this context
  // exported (spx_peer_export: the tableau, the record buffer) is never freed
  // before spx_destroy: the IPC export of a NEW allocation at a freed
  // exported address is not trustworthy on this runtime (round 5: the address
  // and the handle bytes came back, and the peer's first window faulted;
  // profiles/r05/ipc/).  A reload puts them in `pool`, tagged by role, and an
  // allocation of that role takes the smallest pooled buffer that fits, so an
  // exported address is only ever reused by its own allocation (whose handle
  // stays valid).  Sizes are rounded up to a class (<= 12.5 % more), and a
  // role holds at most POOL_MAX buffers: a load needing another fails with
  // SPX_E_STATE instead of growing.  spx_destroy first waits (bounded) for
  // every peer's release mark (close_peers), then frees everything.
  // Every buffer spx_peer_export ever exported stays in `ever_exported`, so a
  // buffer taken from the pool and not exported again (a load whose import
  // was skipped or failed, or an alloc_common that failed after pool_take)
  // still goes back to the pool, never to hipFree.
  std::set<void*> ever_exported;
  bool imported_load = false;   // an spx_peer_import succeeded since the current load
  // the current load's tableau or record buffer is a plain allocation because
  // its role's pool was full (round 6): it is never exported, so this load
  // runs without the peer chain (spx_peer_import returns SPX_E_NOPEER on every
  // rank), and the next load frees it
  bool export_blocked = false;
  uint32_t peer_gen = 0;        // successful IPC imports of this context (the same on every rank)
  struct Pooled {
    void* p;
    size_t bytes;
    int role;                   // POOL_TABLEAU / POOL_RECORDS (its allocation flags follow)
    uint32_t gen;               // records: the import generation whose release marks it
                                // receives (peers write them when they close that mapping);
                                // 0 if it was never imported
  };
  std::vector<Pooled> pool;
  int peer_push = 0;            // leaving-row transport requested for the next import (spx_set_peer_push)
  ChainPeers* d_peers = nullptr;  // device copy of `peers` (the chain kernel's argument)
  int peer_same_dev = 1;        // ranks whose chains share this rank's GPU
  int peer_B = 0, peer_cb = BLK;  // the shard chain's grid, agreed by every rank at import

  // start handshake of persistent chains (spx_chain.hpp chain_start): bound in
  // us (0: automatic, < 0: force ABORT, a test hook), and the windows rerun
  // after a chain found its blocks not co-resident (ST_NOTRES)
  int64_t hs_us = 0;
  int64_t chain_reruns = 0;
  int64_t notres_at = -1;   // the iteration count at the last start-handshake abort
  // peer-only shards: the first of the current run of consecutive aborts, and
  // how long such a run may last before the call gives up (a rank whose host
  // drains late keeps its peers' reruns aborting until it arrives)
  std::chrono::steady_clock::time_point notres_since{};
  double peer_rerun_s = 30.0;
  int64_t rp_target = -1;  // iterations the outstanding spx_run_pivots request ends at (-1: none)
  bool st_fresh = false;   // h_st equals the device State (pulled, nothing enqueued since)

  // graph cache
  // captured launch sequences by chunk (pivots): a few sizes per context
  // (the bench's warmup and timed runs, spx_solve), so none is rebuilt inside
  // a timed region
  // (key: chunk, the window set parity and last_fold the capture began with;
  // value: the graph and the host state its replay leaves: parity, last_fold)
  struct GraphEntry {
    hipGraphExec_t exec;
    int par_after;
    bool fold_after;
  };
  std::map<int64_t, GraphEntry> graphs;
  hipGraphExec_t gexec = nullptr;  // the one build_graph returned last
  // windows per replayed graph (SPX_GRAPH_WINDOWS): consecutive windows in one
  // graph pay one graph-launch gap (8.4 us at config 3) instead of one each
  int graph_windows = 4;

  // elimination timing
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  size_t ev_used = 0;
  // pivot-choice timing (spx_set_chain_timing): events around each window's
  // chain (the persistent kernel, or the lazy kernels of all its slots)
  bool time_chain = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> evc;
  size_t evc_used = 0;
  int64_t touched_at_reset = 0;
};

namespace {

#define HIPC(expr)                                                                  \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess) {                                                         \
      ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
      return SPX_E_HIP;                                                             \
    }                                                                               \
  } while (0)

#define NCCLC(expr)                                                                 \
  do {                                                                              \
    ncclResult_t e_ = (expr);                                                       \
    if (e_ != ncclSuccess) {                                                        \
      ctx->err = std::string(#expr) + ": " + ncclGetErrorString(e_);                \
      return SPX_E_RCCL;                                                            \
    }                                                                               \
  } while (0)

#define CHECK_ARG(cond, msg)                                                        \
  do {                                                                              \
    if (!(cond)) {                                                                  \
      ctx->err = (msg);                                                             \
      return SPX_E_ARG;                                                             \
    }                                                                               \
  } while (0)

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

void drop_graphs(spx_ctx* ctx) {
  for (auto& kv : ctx->graphs) (void)hipGraphExecDestroy(kv.second.exec);
  ctx->graphs.clear();
  ctx->gexec = nullptr;
}

// IPC release marks (spx_ctx::ever_exported): granule {CLOSE_TAG, generation} at
// slot `rank` of each peer's release plane, written through this rank's
// mapping of that peer's record buffer before the mapping is closed.
constexpr unsigned CLOSE_TAG = 0xC105ED00u;
__global__ void peer_release_kernel(const ChainPeers* pe, uint32_t gen) {
  const int d = threadIdx.x;
  if (d < pe->nranks && d != pe->rank && pe->ratio[d])
    g_store<true>((gu64*)pe->ratio[d] + (size_t)CLOSE_PLANE_SHARD * CHAIN_SH_SLOTS + pe->rank,
                  CLOSE_TAG, gen);
}

void close_peers(spx_ctx* ctx) {
  if (!ctx->ipc_open.empty() && ctx->peer_gen > 0 && ctx->d_peers) {
    // release marks first (the peers' record buffers are still mapped)
    hipLaunchKernelGGL(peer_release_kernel, dim3(1), dim3(64), 0, ctx->stream,
                       (const ChainPeers*)ctx->d_peers, ctx->peer_gen);
    (void)hipStreamSynchronize(ctx->stream);
  }
  for (void* p : ctx->ipc_open) (void)hipIpcCloseMemHandle(p);
  ctx->ipc_open.clear();
  ctx->peer_ok = false;
  ctx->peers = ChainPeers{};
  ctx->peer_same_dev = 1;
  ctx->peer_B = 0;
}

// Every peer's release mark for import generation `gen` in the record buffer
// `rec` (one this context exported; peers write the marks through their
// mapping of it when they close that mapping), until `deadline`.  True when
// all arrived.
bool wait_peer_release(spx_ctx* ctx, const unsigned long long* rec, uint32_t gen,
                       std::chrono::steady_clock::time_point deadline) {
  if (ctx->nranks <= 1 || !rec || gen == 0) return true;
  std::vector<unsigned long long> h((size_t)ctx->nranks);
  for (;;) {
    if (hipMemcpy(h.data(), rec + (size_t)CLOSE_PLANE_SHARD * CHAIN_SH_SLOTS,
                  sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost) != hipSuccess)
      return false;
    bool all = true;
    for (int q = 0; q < ctx->nranks; ++q)
      if (q != ctx->rank) all &= (unsigned)(h[q] >> 32) == CLOSE_TAG && (uint32_t)h[q] == gen;
    if (all) return true;
    if (std::chrono::steady_clock::now() > deadline) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

// Frees the loaded tableau's buffers; a tableau or record buffer that was
// ever exported goes to the context's pool instead (spx_ctx::pool), whether or
// not the current load exported it again.
constexpr int POOL_TABLEAU = 0, POOL_RECORDS = 1, POOL_MAX = 4;
int free_buffers(spx_ctx* ctx) {
  drop_graphs(ctx);
  close_peers(ctx);
  if (ctx->A && ctx->ever_exported.count(ctx->A)) {
    ctx->pool.push_back({ctx->A, ctx->A_bytes, POOL_TABLEAU, 0u});
    ctx->A = nullptr;
  }
  if (ctx->gr_ratio && ctx->ever_exported.count(ctx->gr_ratio)) {
    // (peers that imported this load write their release marks into it)
    ctx->pool.push_back({ctx->gr_ratio, ctx->gr_bytes, POOL_RECORDS,
                         ctx->imported_load ? ctx->peer_gen : 0u});
    ctx->gr_ratio = nullptr;
  }
  ctx->imported_load = false;
  ctx->export_blocked = false;
  dfree(ctx->A);
  dfree(ctx->obj);
  dfree(ctx->F);
  dfree(ctx->P);
  dfree(ctx->list);
  dfree(ctx->basis);
  dfree(ctx->hist);
  dfree(ctx->enter_part);
  dfree(ctx->ratio_part);
  dfree(ctx->sendbuf);
  dfree(ctx->recvbuf);
  for (Window& w : ctx->wins) {
    dfree(w.F);
    dfree(w.P);
    dfree(w.r);
    dfree(w.c);
    dfree(w.made);
    dfree(w.nlist);
    dfree(w.rec);
    dfree(w.frt);
    dfree(w.Pf);
  }
  dfree(ctx->wins[0].tag);
  dfree(ctx->wins[0].epoch);
  dfree(ctx->wins[0].fix);
  ctx->wins[1].tag = nullptr;
  ctx->wins[1].epoch = nullptr;
  ctx->wins[1].fix = nullptr;
  ctx->wpar = 0;
  ctx->last_fold = false;
  dfree(ctx->gr_enter);
  dfree(ctx->gr_ratio);
  ctx->loaded = false;
  return SPX_OK;
}

// Size class of a pooled role: up to 1/8 more, in 2 MiB steps at least, so a
// pooled buffer serves the sizes near it.
size_t pool_class(size_t bytes) {
  size_t g = (size_t)2 << 20;
  while ((g << 4) <= bytes) g <<= 1;  // g ~ bytes / 8 .. bytes / 16
  return (bytes + g - 1) / g * g;
}

// A buffer of `role` for `bytes`: the smallest pooled one that fits, else a
// new allocation of the role's class (records of multi-process shards are
// uncached).  *got = its size.  SPX_E_STATE when the role's pool is full.
int pool_take(spx_ctx* ctx, int role, size_t bytes, bool uncached, void** out, size_t* got) {
  int best = -1;
  int held = 0;
  for (int x = 0; x < (int)ctx->pool.size(); ++x) {
    const auto& e = ctx->pool[x];
    if (e.role != role) continue;
    ++held;
    if (e.bytes >= bytes && (best < 0 || e.bytes < ctx->pool[best].bytes)) best = x;
  }
  if (best >= 0) {
    *out = ctx->pool[best].p;
    *got = ctx->pool[best].bytes;
    ctx->pool.erase(ctx->pool.begin() + best);
    return SPX_OK;
  }
  // a full pool: a plain allocation of this load only, which is never exported
  // (and so freed by the next load), instead of growing the pool
  const bool overflow = held >= POOL_MAX;
  if (overflow) ctx->export_blocked = true;
  const size_t sz = overflow ? bytes : pool_class(bytes);
  if (uncached) {
    if (hipExtMallocWithFlags(out, sz, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      HIPC(hipMalloc(out, sz));
    }
  } else {
    HIPC(hipMalloc(out, sz));
  }
  *got = sz;
  return SPX_OK;
}

int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// Elimination geometry: rows per thread R, row chunks rch, column groups G.
void choose_geometry(spx_ctx* ctx) {
  const int64_t m = ctx->m_local;
  ctx->R = (m >= 1024) ? 4 : 2;
  if (ctx->tune_R == 2 || ctx->tune_R == 4 || ctx->tune_R == 8) ctx->R = ctx->tune_R;
  // measured (profiles/r01/tune_m*.log): non-temporal stores win on shards of
  // >= 4096 rows (6.55 TB/s), plain stores on 1024 / 2048-row shards
  ctx->elim_nt = ctx->tune_nt >= 0 ? ctx->tune_nt : (m >= 4096 ? 2 : 0);
  const int64_t rc = (int64_t)BLK * ctx->R;
  ctx->rch = (int)std::max<int64_t>(1, (m + rc - 1) / rc);
  // measured on config 3 (tools/tune_elim.py, profiles/r01/tune_*.log): five
  // resident workgroups per CU streaming interleaved column windows with
  // non-temporal stores (6.6 TB/s) beat a full 8-per-CU grid; a grid that
  // does not fit in one residency round (1536) leaves a tail
  const int target = ctx->tune_wgs > 0 ? ctx->tune_wgs : 1280;
  ctx->G = std::max(1, target / ctx->rch);
  ctx->G = (int)std::min<int64_t>(ctx->G, std::max<int64_t>(1, ctx->N));
  ctx->nbn = (int)std::max<int64_t>(1, (ctx->N + BLK - 1) / BLK);
  ctx->nbr = (int)std::min<int64_t>(256, std::max<int64_t>(1, (m + 2 * BLK - 1) / (2 * BLK)));
}

template <int R, bool NTL, bool NTS, bool ILV, bool PIPE>
void launch_elim_t(spx_ctx* ctx) {
  hipLaunchKernelGGL((elim_kernel<R, NTL, NTS, ILV, PIPE>), dim3(ctx->rch * ctx->G), dim3(BLK),
                     0, ctx->stream, ctx->A, ctx->ld, ctx->m_local, ctx->row0, ctx->N, ctx->F,
                     ctx->P, ctx->list, ctx->rch, ctx->G, ctx->enter_part, ctx->nbn,
                     ctx->ratio_part, ctx->obj, ctx->basis, ctx->prm, ctx->st, ctx->elim_xcd);
}

template <int R, bool ILV, bool PIPE>
void launch_elim_nt(spx_ctx* ctx) {
  switch (ctx->elim_nt & 3) {
    case 0: launch_elim_t<R, false, false, ILV, PIPE>(ctx); break;
    case 1: launch_elim_t<R, true, false, ILV, PIPE>(ctx); break;
    case 2: launch_elim_t<R, false, true, ILV, PIPE>(ctx); break;
    default: launch_elim_t<R, true, true, ILV, PIPE>(ctx); break;
  }
}

template <int R>
void launch_elim_r(spx_ctx* ctx) {
  if (ctx->elim_ilv) {
    if (ctx->elim_pipe) launch_elim_nt<R, true, true>(ctx);
    else launch_elim_nt<R, true, false>(ctx);
  } else {
    if (ctx->elim_pipe) launch_elim_nt<R, false, true>(ctx);
    else launch_elim_nt<R, false, false>(ctx);
  }
}

void launch_elim(spx_ctx* ctx) {
  switch (ctx->R) {
    case 8: launch_elim_r<8>(ctx); break;
    case 4: launch_elim_r<4>(ctx); break;
    default: launch_elim_r<2>(ctx); break;
  }
}

template <int MODE>
void launch_norm(spx_ctx* ctx) {
  hipLaunchKernelGGL((norm_kernel<MODE>), dim3(ctx->nbn), dim3(BLK), 0, ctx->stream, ctx->A,
                     ctx->ld, ctx->m_local, ctx->row0, ctx->N, ctx->obj, ctx->F, ctx->P,
                     ctx->list, ctx->ratio_part, ctx->recvbuf, ctx->gstride, ctx->nranks,
                     ctx->enter_part, ctx->basis, ctx->hist, ctx->prm, ctx->st);
}

void launch_prime(spx_ctx* ctx) {
  hipLaunchKernelGGL(prime_kernel, dim3(ctx->nbr), dim3(BLK), 0, ctx->stream, ctx->A, ctx->ld,
                     ctx->m_local, ctx->row0, ctx->N, ctx->obj, ctx->F, ctx->enter_part,
                     ctx->nbn, ctx->ratio_part, ctx->basis, ctx->prm, ctx->st);
}

constexpr int LOOP_MAX = 16;

int loop_fail(spx_ctx* ctx) {
  ctx->err = "loopback group barrier timed out (a peer rank stopped)";
  return SPX_E_STATE;
}

// Publish on my stream, meet the peers, make my stream wait for theirs.
int loop_meet(spx_ctx* ctx, hipEvent_t spx_ctx::*ev) {
  LoopGroup* G = ctx->loop;
  HIPC(hipEventRecord(ctx->*ev, ctx->stream));
  if (!G->barrier()) return loop_fail(ctx);
  for (int q = 0; q < G->n; ++q) HIPC(hipStreamWaitEvent(ctx->stream, G->members[q]->*ev, 0));
  return SPX_OK;
}

// recvbuf[q] <- sendbuf of rank q, for all q (RCCL, or the in-process group).
int comm_allgather(spx_ctx* ctx) {
  if (ctx->comm) {
    NCCLC(ncclAllGather(ctx->sendbuf, ctx->recvbuf, (size_t)ctx->gstride, ncclUint8, ctx->comm,
                        ctx->stream));
    return SPX_OK;
  }
  LoopGroup* G = ctx->loop;
  int rc = loop_meet(ctx, &spx_ctx::ev_ready);
  if (rc) return rc;
  for (int q = 0; q < G->n; ++q)
    HIPC(hipMemcpyAsync(ctx->recvbuf + q * ctx->gstride, G->members[q]->sendbuf,
                        (size_t)ctx->gstride, hipMemcpyDeviceToDevice, ctx->stream));
  return loop_meet(ctx, &spx_ctx::ev_done);  // peers' sendbuf reusable after this
}

// Record a timing event on the stream; while the stream is being captured,
// insert an event-record node into the capture graph in stream order instead.
int record_event(spx_ctx* ctx, hipEvent_t ev) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIPC(hipStreamIsCapturing(ctx->stream, &cs));
  if (cs != hipStreamCaptureStatusActive) {
    HIPC(hipEventRecord(ev, ctx->stream));
    return SPX_OK;
  }
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  HIPC(hipStreamGetCaptureInfo_v2(ctx->stream, &cs, &id, &g, &deps, &ndeps));
  hipGraphNode_t node;
  HIPC(hipGraphAddEventRecordNode(&node, g, deps, ndeps, ev));
  HIPC(hipStreamUpdateCaptureDependencies(ctx->stream, &node, 1,
                                          hipStreamSetCaptureDependencies));
  return SPX_OK;
}

// entering partial slots: one per wave of the lazy kernels, or one per block of
// the persistent chain (up to CHAIN_MAX_BLOCKS)
int enter_part_len(const spx_ctx* ctx) {
  return std::max(NWAVE * ctx->nbn, CHAIN_MAX_BLOCKS);
}

// ratio partial slots: prime / fused elim / lazy_ratio grids
int ratio_part_len(const spx_ctx* ctx) {
  return std::max({ctx->nbr, ctx->rch, NWAVE * (int)((ctx->m_local + BLK - 1) / BLK)});
}

// flush grid: row chunks of 2*BLK rows x column groups (about target_wgs blocks)
int flush_rch(const spx_ctx* ctx, int rt) {
  return (int)((ctx->m_local + rt * BLK - 1) / (rt * BLK));
}
// column groups: fill the resident capacity (blocks/CU x CUs) once, no tail wave
int flush_groups(spx_ctx* ctx, const void* kern, int rch, int threads = BLK) {
  if (ctx->tune_wgs > 0) return std::max(1, ctx->tune_wgs / rch);
  if (!ctx->n_cu) {
    (void)hipDeviceGetAttribute(&ctx->n_cu, hipDeviceAttributeMultiprocessorCount, ctx->device);
    if (ctx->n_cu <= 0) ctx->n_cu = 256;
  }
  int& bpc = ctx->flush_bpc[kern];
  if (!bpc) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, threads, 0) != hipSuccess || nb < 1)
      nb = 2;
    bpc = nb;
  }
  return std::max(1, bpc * ctx->n_cu / rch);
}
// lazy_ratio grid: one row per thread
int lazy_ratio_grid(const spx_ctx* ctx) {
  return std::max(1, (int)((ctx->m_local + BLK - 1) / BLK));
}

// Persistent chain geometry: B blocks of CB threads (one per CU, all
// resident), each owning <= CB columns and <= CB rows.  Returns B (and CB in
// *cb), or 0 when the chain does not apply (row shards, the launch-per-phase
// mode, or a tableau wider than CB x CUs columns).  mode 2 / 3 force 256- /
// 512-thread blocks; automatic: 256 threads (measured faster than 512 at
// config 3, profiles/r02), 512 when the tableau needs more than 256 blocks.
int device_cus(int device) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      n <= 0)
    n = 256;
  return n;
}

// Threads per chain block for a grid of `wide` columns / rows: 256 (measured
// faster than 512 at config 3, profiles/r02) unless the tableau needs more
// than 256 blocks of them; chain modes 2 / 3 force 256 / 512.
int chain_cb(int mode, int64_t wide, int n_cu) {
  return mode == 2 ? 256 : mode == 3 ? 512
         : (wide > 256 * std::min(n_cu, CHAIN_MAX_BLOCKS) ? 512 : 256);
}

// Blocks of a chain of cb threads over N columns and `rows` rows: the N-1
// candidate columns set the width (the RHS column rides along with the last
// block's last thread when B * cpb == N - 1, spx_chain.hpp xown).
int64_t chain_need(int64_t N, int64_t rows, int cb, int min_blocks) {
  return std::max<int64_t>({(N - 1 + cb - 1) / cb, (rows + cb - 1) / cb, 1, (int64_t)min_blocks});
}

// Persistent chain geometry: B blocks of CB threads (one per CU, all
// resident), each owning <= CB columns and <= CB rows.  Returns B (and CB in
// *cb), or 0 when the chain does not apply (the launch-per-phase mode, a
// refused admission, or a tableau wider than CB x CUs columns).  Row shards
// take the geometry every rank agreed on at spx_peer_import /
// spx_peer_chain_local (shard_geometry), so no rank decides alone.
// Persistent chain geometry: B blocks of CB threads (one per CU, all
// resident), each owning <= CB columns and <= CB rows.  Returns B (and CB in
// *cb), or 0 when the chain does not apply (the launch-per-phase mode, a
// refused admission, or a tableau wider than CB x CUs columns).  Row shards
// take the geometry every rank agreed on at spx_peer_import /
// spx_peer_chain_local (shard_geometry), so no rank decides alone.
int chain_blocks(spx_ctx* ctx, int* cb_out = nullptr, bool ignore_admission = false) {
  if (ctx->chain_mode == 1) return 0;
  if (ctx->sharded) {  // shards: only once the peers are known
    if (!ctx->peer_ok) return 0;
    if (cb_out) *cb_out = ctx->peer_cb;
    return ctx->chain_denied ? 0 : ctx->peer_B;
  }
  if (ctx->chain_denied && !ignore_admission) return 0;
  if (!ctx->n_cu) ctx->n_cu = device_cus(ctx->device);
  const int cb = chain_cb(ctx->chain_mode, std::max<int64_t>(ctx->N, ctx->m_local), ctx->n_cu);
  if (cb_out) *cb_out = cb;
  const int64_t need = chain_need(ctx->N, ctx->m_local, cb, ctx->chain_min_blocks);
  const int64_t cap = std::min<int64_t>((int64_t)ctx->n_cu, CHAIN_MAX_BLOCKS);
  return need <= cap ? (int)need : 0;
}

// ---- admission of persistent chains ("Admission") ----------
// A persistent chain needs all of its B blocks resident at once (one per CU:
// its LDS pin), and the chains of every context on a device share the CUs.
// The process counts, per device, the blocks of the chains it has in flight; a
// call whose chain would push that sum over the budget (default: the device's
// CU count; SPX_CHAIN_BUDGET or spx_set_chain_budget override it) runs its
// windows with the launch-per-phase chain instead, which is bit-identical and
// needs no co-residency.  So concurrent /solve calls slow down instead of
// timing out.
//
// Across processes (gunicorn's two workers, /root/reference/dockerfile:34)
// the budget is shared through a table in /dev/shm/spx_chain_<PCI bus id>: 64
// entries {pid, blocks, start time}, read and written under flock.  Each process keeps
// its entry equal to its in-flight blocks on that GPU; a chain is admitted
// only when every live process's blocks plus its own fit the budget.  Entries
// of dead processes (kill(pid, 0) -> ESRCH) count as free, and a process
// clears its entries at exit.  SPX_CHAIN_SHM=0 turns the table off (the
// process-local count still applies); the start handshake (chain_start) is
// the backstop for GPU users outside this scheme.
constexpr int SHM_SLOTS = 64;
struct ShmEntry {
  int32_t pid, blocks;
  uint64_t start;  // the process's start time (/proc/<pid>/stat): a reused pid is not it
};
static_assert(sizeof(ShmEntry) == 16, "the table's on-disk entry");

// Start time of a live process in clock ticks since boot (0: unknown).
uint64_t proc_start(int32_t pid) {
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
  FILE* f = std::fopen(path, "r");
  if (!f) return 0;
  char buf[1024];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* p = std::strrchr(buf, ')');  // the command name may hold spaces
  if (!p) return 0;
  // fields after the name: state (3) ... starttime (22)
  int field = 2;
  for (++p; *p && field < 22; ++p)
    if (*p == ' ') ++field;
  return field == 22 ? std::strtoull(p, nullptr, 10) : 0;
}

// This process's start time (read once; a fork()ed child reads its own).
uint64_t my_start() {
  static pid_t who = 0;
  static uint64_t t = 0;
  const pid_t me = getpid();
  if (who != me) {
    t = proc_start((int32_t)me);
    who = me;
  }
  return t;
}

// Is the table entry's process alive (and the same process that wrote it)?
bool shm_entry_live(const ShmEntry& e) {
  if (!(kill(e.pid, 0) == 0 || errno == EPERM)) return false;
  const uint64_t st = proc_start(e.pid);
  return e.start == 0 || st == 0 || st == e.start;
}

struct ShmTable {
  int fd = -1;
  pid_t opener = 0;  // fds inherited across fork() share their flock: reopen
  std::string path;
};

std::string shm_path(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, device) != hipSuccess)
    std::snprintf(bus, sizeof(bus), "dev%d", device);
  std::string p = "/dev/shm/spx_chain_";
  for (const char* c = bus; *c; ++c) p += std::isalnum((unsigned char)*c) ? *c : '_';
  return p;
}

struct ChainAdmission {
  std::mutex mu;
  std::map<int, int> used;    // chain blocks in flight, by device
  std::map<int, int> budget;  // explicit budgets (spx_set_chain_budget)
  std::map<int, ShmTable> shm;
  std::set<spx_ctx*> deferred;  // contexts with reservations waiting for their adm_ev
  ~ChainAdmission();
};
ChainAdmission& adm() {
  static ChainAdmission a;
  return a;
}

bool shm_enabled() {
  const char* e = std::getenv("SPX_CHAIN_SHM");
  return !(e && e[0] == '0');
}

// The device's table, opened by this process (-1: unavailable).
int shm_fd_locked(ChainAdmission& a, int device) {
  ShmTable& t = a.shm[device];
  if (t.fd >= 0 && t.opener == getpid()) return t.fd;
  if (t.fd >= 0) close(t.fd);  // inherited across fork(): its flock is the parent's
  t.fd = -1;
  if (!shm_enabled()) return -1;
  if (t.path.empty()) t.path = shm_path(device);
  // (no symlink followed; only a regular file is used as the table)
  t.fd = open(t.path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC | O_NOFOLLOW, 0666);
  struct stat sb;
  if (t.fd >= 0 && (fstat(t.fd, &sb) != 0 || !S_ISREG(sb.st_mode))) {
    close(t.fd);
    t.fd = -1;
  }
  // every process (user) on the GPU shares the table: 0666 regardless of the
  // umask (fchmod, not a process-wide umask change; fails harmlessly when
  // another user created the file)
  if (t.fd >= 0) (void)fchmod(t.fd, 0666);
  t.opener = getpid();
  return t.fd;
}

// Under the table's flock, in one critical section: the blocks of every OTHER
// live process; then, if `admit` says those plus this process's own fit
// (admit == nullptr: always), this process's entry set to `mine` (mine < 0:
// read only).  Returns the others' blocks, or -1 when the table is
// unavailable (the process-local count then decides alone); *ok the verdict.
template <typename Admit>
int shm_exchange(int fd, int mine, Admit admit, bool* ok = nullptr) {
  if (ok) *ok = true;
  if (fd < 0) return -1;
  if (flock(fd, LOCK_EX) != 0) return -1;
  ShmEntry e[SHM_SLOTS];
  std::memset(e, 0, sizeof(e));
  const ssize_t got = pread(fd, e, sizeof(e), 0);
  (void)got;  // (a short or new file reads as free entries)
  const int32_t me = (int32_t)getpid();
  int64_t others = 0;  // (entries are untrusted: each clamped, summed in 64 bits)
  int slot = -1, free_slot = -1;
  bool dirty = false;
  for (int x = 0; x < SHM_SLOTS; ++x) {
    if (e[x].pid == me) {
      slot = x;
    } else if (e[x].pid > 0 && e[x].blocks > 0) {
      if (shm_entry_live(e[x])) {
        others += std::min<int64_t>(e[x].blocks, CHAIN_MAX_BLOCKS);
      } else {  // a dead process's entry (or its pid reused): free it
        e[x] = ShmEntry{0, 0, 0};
        dirty = true;
      }
    }
    if (free_slot < 0 && (e[x].pid <= 0 || e[x].blocks <= 0) && e[x].pid != me) free_slot = x;
  }
  const bool go = admit((int)std::min<int64_t>(others, INT32_MAX / 2));
  if (ok) *ok = go;
  if (go && mine >= 0) {
    if (slot < 0) slot = free_slot;
    if (slot >= 0) {
      e[slot] = mine > 0 ? ShmEntry{me, mine, my_start()} : ShmEntry{0, 0, 0};
      dirty = true;
    }
  }
  if (dirty) (void)!pwrite(fd, e, sizeof(e), 0);
  flock(fd, LOCK_UN);
  return (int)std::min<int64_t>(others, INT32_MAX / 2);
}
int shm_set(int fd, int mine) {
  return shm_exchange(fd, mine, [](int) { return true; });
}

ChainAdmission::~ChainAdmission() {
  // normal exit: this process's entries go back to the tables
  for (auto& kv : shm)
    if (kv.second.fd >= 0 && kv.second.opener == getpid()) (void)shm_set(kv.second.fd, 0);
}

int adm_budget_locked(ChainAdmission& a, const spx_ctx* ctx) {
  const auto it = a.budget.find(ctx->device);
  if (it != a.budget.end()) return it->second;
  if (const char* e = std::getenv("SPX_CHAIN_BUDGET")) return std::max(0, std::atoi(e));
  return ctx->n_cu;
}

void adm_settle_locked(ChainAdmission& a, spx_ctx* ctx, bool drained);

// Decide the chain of the call starting now.  Returns true when the call holds
// a reservation, which adm_release must return once the call's launches ran.
bool adm_acquire(spx_ctx* ctx) {
  const bool was = ctx->chain_denied;
  ctx->chain_denied = false;
  const int B = ctx->win_k ? chain_blocks(ctx, nullptr, true) : 0;
  if (B <= 0) return false;  // no persistent chain for this call anyway
  ChainAdmission& a = adm();
  bool ok;
  {
    std::lock_guard<std::mutex> lk(a.mu);
    // reservations whose launches have run (deferred by calls that did not
    // wait for them), this context's and every other's in the process
    for (auto it = a.deferred.begin(); it != a.deferred.end();) {
      spx_ctx* d = *it++;  // (adm_settle_locked may erase d)
      adm_settle_locked(a, d, false);
    }
    const int cap = adm_budget_locked(a, ctx);
    int& used = a.used[ctx->device];
    const int extra = std::max(0, B - ctx->adm_blocks);  // 0: this context holds B already
    // row shards must all take the same chain: never refused,
    // but their blocks count against the device's budget while they run, so
    // single-GPU chains beside them are refused instead of over-subscribing
    ok = ctx->sharded || used + extra <= cap;
    if (ok && extra > 0) {  // the other processes' chains on this GPU (the shared table):
      // read and claim under ONE flock, so two processes cannot both fit
      const bool force = ctx->sharded;
      const int want = used + extra;
      (void)shm_exchange(shm_fd_locked(a, ctx->device), want,
                         [&](int others) { return force || others + want <= cap; }, &ok);
    }
    if (ok) {
      used += extra;
      ctx->adm_blocks += extra;
      ctx->adm_calls++;
    }
  }
  ctx->chain_denied = !ok;
  ctx->chain_calls[ok ? 0 : 1]++;
  if (ctx->chain_denied != was) drop_graphs(ctx);  // the cached graph has the other chain
  return ok;
}

void adm_release_locked(ChainAdmission& a, spx_ctx* ctx) {
  if (ctx->adm_calls > 0 && --ctx->adm_calls == 0) {
    int& used = a.used[ctx->device];
    used -= ctx->adm_blocks;
    if (ctx->adm_blocks > 0) (void)shm_set(shm_fd_locked(a, ctx->device), used);
    ctx->adm_blocks = 0;
  }
}

void adm_release(spx_ctx* ctx) {
  ChainAdmission& a = adm();
  std::lock_guard<std::mutex> lk(a.mu);
  adm_release_locked(a, ctx);
}

// Release a context's deferred reservations once their launches have run:
// `drained` (its stream was just synchronised) or its adm_ev has completed.
void adm_settle_locked(ChainAdmission& a, spx_ctx* ctx, bool drained) {
  if (ctx->adm_deferred == 0) return;
  if (!drained && (!ctx->adm_ev || hipEventQuery(ctx->adm_ev) != hipSuccess)) return;
  for (; ctx->adm_deferred > 0; --ctx->adm_deferred) adm_release_locked(a, ctx);
  a.deferred.erase(ctx);
}
void adm_settle(spx_ctx* ctx, bool drained) {
  ChainAdmission& a = adm();
  std::lock_guard<std::mutex> lk(a.mu);
  adm_settle_locked(a, ctx, drained);
}

// Holds a call's reservation: released at once when the call drained its
// stream, else deferred behind an event recorded after the call's launches
// and released by the first of: a drain of the context (spx_sync, a State
// pull, spx_destroy), its next call, or any admission decision in the process
// that finds the event complete.  (A host callback on the stream did the same
// promptly, but cost every call ~46 us of stream time: tools/dbg/call_overhead.py.)
struct AdmCall {
  spx_ctx* ctx;
  bool held = false;
  bool drained = false;
  explicit AdmCall(spx_ctx* c) : ctx(c) {}
  ~AdmCall() {
    if (!held) return;
    if (!drained && !ctx->adm_ev &&
        hipEventCreateWithFlags(&ctx->adm_ev, hipEventDisableTiming) != hipSuccess)
      ctx->adm_ev = nullptr;
    if (drained || !ctx->adm_ev || hipEventRecord(ctx->adm_ev, ctx->stream) != hipSuccess) {
      adm_release(ctx);
      return;
    }
    ChainAdmission& a = adm();
    std::lock_guard<std::mutex> lk(a.mu);
    ctx->adm_deferred++;
    a.deferred.insert(ctx);
  }
};

// An event pair from the context's pool (created on first use).
int next_event_pair(spx_ctx* ctx, std::vector<std::pair<hipEvent_t, hipEvent_t>>& pool,
                    size_t& used, std::pair<hipEvent_t, hipEvent_t>** out) {
  if (used == pool.size()) {
    hipEvent_t a, b;
    HIPC(hipEventCreate(&a));
    HIPC(hipEventCreate(&b));
    pool.emplace_back(a, b);
  }
  *out = &pool[used++];
  return SPX_OK;
}

// The gated row_fix of window set `sid` (the row_fix fold):
// rewrites its leaving rows only if that set's fold chain left them owed.
template <int KMAX>
void launch_gated_fix_t(spx_ctx* ctx, int sid) {
  hipLaunchKernelGGL((row_fix_kernel<KMAX, BLK, true>), dim3(ctx->nbn), dim3(BLK), 0,
                     ctx->stream, ctx->A, ctx->ld, ctx->m_local, ctx->row0, ctx->N,
                     ctx->wins[sid], KMAX);
}
void launch_gated_fix(spx_ctx* ctx, int sid) {
  switch (ctx->win_k) {
    case 2: return launch_gated_fix_t<2>(ctx, sid);
    case 4: return launch_gated_fix_t<4>(ctx, sid);
    case 8: return launch_gated_fix_t<8>(ctx, sid);
    case 12: return launch_gated_fix_t<12>(ctx, sid);
    case 16: return launch_gated_fix_t<16>(ctx, sid);
    case 24: return launch_gated_fix_t<24>(ctx, sid);
    case 28: return launch_gated_fix_t<28>(ctx, sid);
    default: return launch_gated_fix_t<32>(ctx, sid);
  }
}

// The end of a call's enqueued windows (and before anything reads or changes
// the tableau outside the windows): the last window, if a fold window, owes
// its leaving rows' fix -- settle it on the stream.
int settle_fold(spx_ctx* ctx) {
  if (!ctx->last_fold) return SPX_OK;
  launch_gated_fix(ctx, ctx->wpar ^ 1);
  ctx->last_fold = false;
  HIPC(hipGetLastError());
  return SPX_OK;
}

template <int KMAX>
int enqueue_window_t(spx_ctx* ctx, int npiv, bool time_flush) {
  const int nbw = lazy_ratio_grid(ctx);
  int cb = BLK;
  const int B = chain_blocks(ctx, &cb);
  // this window's buffer set and the previous window's (the host's parity)
  const int S = ctx->wpar, P = S ^ 1;
  const Window& win = ctx->wins[S];
  // the row_fix fold: the persistent single-GPU chain with
  // 256-thread blocks resolves the previous window's leaving rows itself
  const bool fold = ctx->fold && B > 0 && !ctx->sharded && cb == 256;
  // a window that is not a fold window reads a tableau whose leaving rows are
  // all fixed: settle what the last fold window owes first
  if (!fold && ctx->last_fold) launch_gated_fix(ctx, P);
  std::pair<hipEvent_t, hipEvent_t>* ec = nullptr;
  if (ctx->time_chain) {
    int rc = next_event_pair(ctx, ctx->evc, ctx->evc_used, &ec);
    if (!rc) rc = record_event(ctx, ec->first);
    if (rc) return rc;
  }
  if (B > 0) {
    const int cpb = (int)((ctx->N - 1 + B - 1) / B);  // (B * cpb == N-1: xown owns the RHS)
    const int rpb = (int)std::max<int64_t>(1, (ctx->m_local + B - 1) / B);
    auto kern = ctx->sharded ? (cb == 512 ? chain_shard_kernel<KMAX, 512>
                                          : chain_shard_kernel<KMAX, 256>)
                : fold ? chain_kernel<KMAX, 256, true>
                       : (cb == 512 ? chain_kernel<KMAX, 512> : chain_kernel<KMAX, 256>);
    hipLaunchKernelGGL(kern, dim3(B), dim3(cb), 0, ctx->stream, ctx->enter_part, ctx->st,
                       (const Params*)ctx->prm, std::max(NWAVE * ctx->nbn, B),
                       (const double*)ctx->A, ctx->ld, ctx->m_local, ctx->N, ctx->obj, win,
                       npiv, ctx->basis, ctx->hist, ctx->gr_enter, ctx->gr_ratio, cpb, rpb,
                       (const ChainPeers*)ctx->d_peers, ctx->wins[P], 0, ctx->A);
  } else if (ctx->sharded && !ctx->comm && !ctx->loop) {
    ctx->err = "a peer-only shard needs the persistent chain (windowed, spx_peer_import done, "
               "chain mode != 1, and its grid fits)";
    return SPX_E_STATE;
  }
  for (int q = 0; B == 0 && q < npiv; ++q) {
    hipLaunchKernelGGL(lazy_ratio_kernel<KMAX>, dim3(nbw), dim3(BLK), 0, ctx->stream,
                       (const Key*)ctx->enter_part, ctx->st, (const Params*)ctx->prm,
                       NWAVE * ctx->nbn, q, (const double*)ctx->A, ctx->ld, ctx->m_local,
                       ctx->row0, ctx->N, (const double*)ctx->obj, win, ctx->ratio_part,
                       (const int64_t*)ctx->basis);
    if (!ctx->sharded) {
      hipLaunchKernelGGL(lazy_norm_kernel<KMAX>, dim3(ctx->nbn), dim3(BLK), 0, ctx->stream,
                         (const Key*)ctx->ratio_part, ctx->st, (const Params*)ctx->prm,
                         NWAVE * nbw, q, (const double*)ctx->A, ctx->ld, ctx->m_local,
                         ctx->row0, ctx->N, ctx->obj, win, npiv - 1, ctx->enter_part,
                         ctx->basis, ctx->hist, nullptr, (int64_t)0, 0);
    } else {
      // row shard: local candidate row (current values) -> ONE all-gather of
      // [key | p] -> every rank takes the winner's p
      hipLaunchKernelGGL(lazy_prep_kernel<KMAX>, dim3(ctx->nbn), dim3(BLK), 0, ctx->stream,
                         (const Key*)ctx->ratio_part, (const State*)ctx->st,
                         (const Params*)ctx->prm, NWAVE * nbw, q, (const double*)ctx->A,
                         ctx->ld, ctx->m_local, ctx->row0, ctx->N, win, ctx->sendbuf,
                         ctx->rank, (const int32_t*)ctx->d_stop);
      const int rc = comm_allgather(ctx);
      if (rc) return rc;
      hipLaunchKernelGGL((lazy_norm_kernel<KMAX, true>), dim3(ctx->nbn), dim3(BLK), 0,
                         ctx->stream, (const Key*)ctx->ratio_part, ctx->st,
                         (const Params*)ctx->prm, NWAVE * nbw, q, (const double*)ctx->A,
                         ctx->ld, ctx->m_local, ctx->row0, ctx->N, ctx->obj, win,
                         npiv - 1, ctx->enter_part, ctx->basis, ctx->hist,
                         (const char*)ctx->recvbuf, ctx->gstride, ctx->nranks);
    }
  }
  if (ec) {
    const int rc = record_event(ctx, ec->second);
    if (rc) return rc;
  }
  // A timed flush outside a capture carries its events in its own launch
  // (hipExtLaunchKernel: the events take the kernel's dispatch start / end
  // timestamps, the span rocprofv3 reports, and no event packets sit between
  // the chain and the flush); inside a capture, event-record nodes around it.
  std::pair<hipEvent_t, hipEvent_t>* e = nullptr;
  bool ext = false;
  if (time_flush) {
    int rc = next_event_pair(ctx, ctx->ev, ctx->ev_used, &e);
    if (rc) return rc;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIPC(hipStreamIsCapturing(ctx->stream, &cs));
    ext = cs != hipStreamCaptureStatusActive;
    if (!ext && (rc = record_event(ctx, e->first))) return rc;
  }
  auto go = [&](auto kern, int rt, int threads = BLK) {
    const int rch = flush_rch(ctx, rt);
    const int G = flush_groups(ctx, (const void*)kern, rch, threads);
    ctx->last_flush_G = G;
    ctx->last_flush_rch = rch;
    if (ext)
      hipExtLaunchKernelGGL(kern, dim3(rch * G), dim3(threads), 0, ctx->stream, e->first,
                            e->second, 0, ctx->A, ctx->ld, ctx->m_local, ctx->row0, ctx->N, win,
                            npiv, rch, G, (const Params*)ctx->prm, ctx->st,
                            ctx->flush_map | ctx->flush_tail << 8);
    else
      hipLaunchKernelGGL(kern, dim3(rch * G), dim3(threads), 0, ctx->stream, ctx->A, ctx->ld,
                         ctx->m_local, ctx->row0, ctx->N, win, npiv, rch, G, ctx->prm,
                         ctx->st, ctx->flush_map | ctx->flush_tail << 8);
  };
  const bool nts = (ctx->elim_nt & 2) != 0;
  // the LDS-DMA ring of 12 columns per wave over the window's compacted
  // records (the register-ring and dynamically claimed flushes
  // measured slower in rounds 1-2 and were removed)
  if (npiv < KMAX)  // the last window of a request: every slot guarded
    nts ? go(flush_lds_kernel<KMAX, 12, true, true>, 2) : go(flush_lds_kernel<KMAX, 12, false, true>, 2);
  else
    nts ? go(flush_lds_kernel<KMAX, 12, true>, 2) : go(flush_lds_kernel<KMAX, 12, false>, 2);
  if (e && !ext) {
    const int rc = record_event(ctx, e->second);
    if (rc) return rc;
  }
  // the fast-path columns' leaving rows (every window: partial ones included);
  // a tail inside the flush measured 226 vs 182 us
  // (profiles/r03/ab_flush_tail_vs_rowfix.jsonl).  A fold window leaves them
  // to the next fold chain (or the gated row_fix of settle_fold).
  if (!fold)
    hipLaunchKernelGGL(row_fix_kernel<KMAX>, dim3(ctx->nbn), dim3(BLK), 0, ctx->stream, ctx->A,
                       ctx->ld, ctx->m_local, ctx->row0, ctx->N, win, npiv);
  ctx->last_fold = fold;
  ctx->wpar = P;
  HIPC(hipGetLastError());
  return SPX_OK;
}

// Enqueue one window of npiv (<= win_k) pivots followed by its flush.
int enqueue_window(spx_ctx* ctx, int npiv, bool time_flush) {
  switch (ctx->win_k) {
    case 2: return enqueue_window_t<2>(ctx, npiv, time_flush);
    case 4: return enqueue_window_t<4>(ctx, npiv, time_flush);
    case 8: return enqueue_window_t<8>(ctx, npiv, time_flush);
    case 12: return enqueue_window_t<12>(ctx, npiv, time_flush);
    case 16: return enqueue_window_t<16>(ctx, npiv, time_flush);
    case 24: return enqueue_window_t<24>(ctx, npiv, time_flush);
    case 28: return enqueue_window_t<28>(ctx, npiv, time_flush);
    default: return enqueue_window_t<32>(ctx, npiv, time_flush);
  }
}

// Enqueue one pivot (all launches on ctx->stream; no host synchronisation).
int enqueue_pivot(spx_ctx* ctx, bool time_elim) {
  if (!ctx->sharded) {
    launch_norm<MODE_FUSED>(ctx);
  } else {
    hipLaunchKernelGGL(prep_kernel, dim3(ctx->nbn), dim3(BLK), 0, ctx->stream, ctx->A, ctx->ld,
                       ctx->m_local, ctx->row0, ctx->N, ctx->F, ctx->ratio_part, ctx->sendbuf,
                       ctx->rank, ctx->st, (const int32_t*)ctx->d_stop);
    int rc = comm_allgather(ctx);
    if (rc) return rc;
    launch_norm<MODE_FINISH>(ctx);
  }
  if (time_elim) {
    if (ctx->ev_used == ctx->ev.size()) {
      hipEvent_t a, b;
      HIPC(hipEventCreate(&a));
      HIPC(hipEventCreate(&b));
      ctx->ev.emplace_back(a, b);
    }
    auto& e = ctx->ev[ctx->ev_used++];
    int rc = record_event(ctx, e.first);
    if (rc) return rc;
    launch_elim(ctx);
    if ((rc = record_event(ctx, e.second))) return rc;
  } else {
    launch_elim(ctx);
  }
  HIPC(hipGetLastError());
  return SPX_OK;
}

// npiv pivots in the context's mode: one window (<= win_k pivots) + its flush,
// or npiv fused single-pivot steps.  `time_k` > 0 brackets eliminations (or
// flushes) with events: every time_k-th elimination / window.
int enqueue_pivots(spx_ctx* ctx, int npiv, int time_k, int64_t first = 0) {
  if (ctx->win_k) {  // consecutive windows of win_k pivots (the last may be shorter)
    for (int done = 0; done < npiv;) {
      const int n = std::min(ctx->win_k, npiv - done);
      const int rc =
          enqueue_window(ctx, n, time_k > 0 && ((first + done) / ctx->win_k) % time_k == 0);
      if (rc) return rc;
      done += n;
    }
    return SPX_OK;
  }
  for (int i = 0; i < npiv; ++i) {
    const int rc = enqueue_pivot(ctx, time_k > 0 && (first + i) % time_k == 0);
    if (rc) return rc;
  }
  return SPX_OK;
}

int make_params(spx_ctx* ctx, const spx_opts* o, Params* out) {
  spx_opts d;
  spx_default_opts(&d);
  if (!o) o = &d;
  CHECK_ARG(o->rule == SPX_RULE_DANTZIG || o->rule == SPX_RULE_BLAND, "unknown pivot rule");
  Params& p = *out;
  p.rule = o->rule;
  p.skip_zero = o->skip_zero_cols ? 1 : 0;
  p.eps_opt = o->eps_opt;
  p.eps_piv = o->eps_piv;
  p.n_enter = (o->n_enter > 0) ? std::min<int64_t>(o->n_enter, ctx->N - 1) : ctx->N - 1;
  p.iter_limit = (o->max_iters > 0) ? ctx->h_st->iters + o->max_iters : INT64_MAX;
  return SPX_OK;
}

// Start-handshake bound of persistent chains, in s_memrealtime ticks (100 MHz):
// 20 us on one GPU (the grid's blocks are dispatched together), 100 ms for row
// shards (the ranks' hosts enqueue their windows independently, so a rank's
// chain may start that much after another's); spx_set_chain_handshake
// overrides it (< 0: every persistent window aborts, a test hook).
int64_t hs_ticks(const spx_ctx* ctx) {
  if (ctx->hs_us < 0) return ctx->hs_us;  // -k: abort every k-th window (chain_start; test hook)
  if (ctx->hs_us > 0) return ctx->hs_us * 100;
  return ctx->sharded ? 10000000 : 2000;
}

// Host-side writes of State fields (synchronous; between pivot calls only).
int set_state_fields(spx_ctx* ctx, int32_t status, int64_t fc, int64_t fr) {
  ctx->h_st->status = status;
  ctx->h_st->forced_c = fc;
  ctx->h_st->forced_r = fr;
  ctx->h_st->hs_ticks = hs_ticks(ctx);
  HIPC(hipMemcpyAsync(ctx->st, ctx->h_st, sizeof(State), hipMemcpyHostToDevice, ctx->stream));
  return SPX_OK;
}

int rp_recover(spx_ctx* ctx);
int pull_state(spx_ctx* ctx) {
  if (ctx->rp_target >= 0) {  // an spx_run_pivots request may need its rerun first
    const int rc = rp_recover(ctx);
    if (rc) return rc;
  }
  ctx->st_fresh = false;
  HIPC(hipMemcpyAsync(ctx->h_st, ctx->st, sizeof(State), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  ctx->st_fresh = true;
  adm_settle(ctx, true);
  return SPX_OK;
}

// Prepare a pivot call: params, status RUNNING, fresh entering partials and
// the primed first pivot (rule-chosen, or the forced (fr, fc) of spx_pivot_at).
int begin_call(spx_ctx* ctx, const spx_opts* o, AdmCall* adm_call, int64_t fc = -1,
               int64_t fr = -1) {
  if (!ctx->loaded) {
    ctx->err = "no tableau loaded";
    return SPX_E_STATE;
  }
  HIPC(hipSetDevice(ctx->device));
  (void)hipGetLastError();  // drop a stale error of an unrelated earlier call
  int rc = SPX_OK;
  // the host's State copy must be current (iters, status); a pull is a
  // stream round trip, skipped when nothing was enqueued since the last one
  if (!ctx->st_fresh && (rc = pull_state(ctx))) return rc;
  if (ctx->h_stop) __atomic_store_n(ctx->h_stop, 0, __ATOMIC_SEQ_CST);  // (stream drained above)
  Params p;
  if ((rc = make_params(ctx, o, &p))) return rc;
  ctx->st_fresh = false;  // (from here on the device State moves on)
  ctx->h_st->status = ST_RUNNING;
  ctx->h_st->forced_c = fc;
  ctx->h_st->forced_r = fr;
  ctx->h_st->hs_ticks = hs_ticks(ctx);
  // params + State fields (+ the window kernels' entering partials past the
  // nbn that INIT writes) in one launch
  const int n = ctx->win_k ? enter_part_len(ctx) - ctx->nbn : 0;
  hipLaunchKernelGGL(call_begin_kernel, dim3(std::max(1, (n + BLK - 1) / BLK)), dim3(BLK), 0,
                     ctx->stream, ctx->prm, p, ctx->st, (int32_t)ST_RUNNING, fc, fr,
                     ctx->h_st->hs_ticks, ctx->enter_part + ctx->nbn, n);
  launch_norm<MODE_INIT>(ctx);
  if (!ctx->win_k) launch_prime(ctx);
  HIPC(hipGetLastError());
  adm_call->held = adm_acquire(ctx);  // persistent or launch-per-phase chain for this call
  return SPX_OK;
}

// The captured graph of `chunk` pivots for the current host window state (the
// next window's buffer set, and whether the last window was a fold window):
// its launches bake in the sets they use, so each state has its own graph.
int64_t graph_key(const spx_ctx* ctx, int chunk, int par, bool fold) {
  return ((int64_t)chunk << 2) | (par << 1) | (fold ? 1 : 0);
}
int build_graph_for(spx_ctx* ctx, int chunk, int par, bool fold) {
  const auto it = ctx->graphs.find(graph_key(ctx, chunk, par, fold));
  if (it != ctx->graphs.end()) {
    ctx->gexec = it->second.exec;
    return SPX_OK;
  }
  ctx->gexec = nullptr;
  // capture from that state; the host state returns to where it was (the
  // graph's launches advance it, launch_graph)
  const int par0 = ctx->wpar;
  const bool fold0 = ctx->last_fold;
  ctx->wpar = par;
  ctx->last_fold = fold;
  hipGraph_t g = nullptr;
  HIPC(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
  int rc = enqueue_pivots(ctx, chunk, 0);
  hipError_t e = hipStreamEndCapture(ctx->stream, &g);
  const spx_ctx::GraphEntry ge{nullptr, ctx->wpar, ctx->last_fold};
  ctx->wpar = par0;
  ctx->last_fold = fold0;
  if (rc) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) {
    ctx->err = std::string("hipStreamEndCapture: ") + hipGetErrorString(e);
    return SPX_E_HIP;
  }
  e = hipGraphInstantiate(&ctx->gexec, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    ctx->gexec = nullptr;
    ctx->err = std::string("hipGraphInstantiate: ") + hipGetErrorString(e);
    return SPX_E_HIP;
  }
  spx_ctx::GraphEntry en = ge;
  en.exec = ctx->gexec;
  ctx->graphs[graph_key(ctx, chunk, par, fold)] = en;
  return SPX_OK;
}
// The graph for the current state (built when missing).
int build_graph(spx_ctx* ctx, int chunk) {
  return build_graph_for(ctx, chunk, ctx->wpar, ctx->last_fold);
}
// Every state's graph of `chunk`, so none is captured inside a timed region
// (whatever windows were launched directly before it).
int build_graphs_all(spx_ctx* ctx, int chunk) {
  if (!ctx->win_k) return build_graph(ctx, chunk);  // (single pivots: no window state)
  for (int par = 0; par < 2; ++par)
    for (int f = 0; f < (ctx->fold || ctx->last_fold ? 2 : 1); ++f)
      if (const int rc = build_graph_for(ctx, chunk, par, f != 0)) return rc;
  return SPX_OK;
}
// Replay the graph of `chunk` for the current state and advance the state.
int launch_graph(spx_ctx* ctx, int chunk) {
  if (const int rc = build_graph(ctx, chunk)) return rc;
  const auto& en = ctx->graphs[graph_key(ctx, chunk, ctx->wpar, ctx->last_fold)];
  HIPC(hipGraphLaunch(en.exec, ctx->stream));
  ctx->wpar = en.par_after;
  ctx->last_fold = en.fold_after;
  return SPX_OK;
}

int map_status(int32_t st) {
  switch (st) {
    case ST_OPTIMAL: return SPX_OPTIMAL;
    case ST_UNBOUNDED: return SPX_UNBOUNDED;
    case ST_LIMIT: return SPX_ITER_LIMIT;
    case ST_FAULT:
    case ST_NOTRES: return SPX_E_STATE;
    default: return SPX_RUNNING;
  }
}

bool is_fault(int32_t st) { return st == ST_FAULT || st == ST_NOTRES; }

// The device reported a fault (an in-launch exchange timed out), or a window
// that did not run (ST_NOTRES) where the call could not rerun it.
int fault(spx_ctx* ctx) {
  if (ctx->h_st->status == ST_NOTRES)
    ctx->err = "a persistent chain's blocks were not co-resident, so its window did not run "
               "and could not be rerun";
  else
    ctx->err = "device fault: a pivot-chain exchange timed out";
  return SPX_E_STATE;
}

// Reruns of a window whose persistent chain aborted at its start handshake
// before a peer-only shard (no launch-per-phase path) gives up.
constexpr int NOTRES_RETRIES = 16;

// A persistent chain found its blocks not co-resident (ST_NOTRES, spx_chain.hpp
// chain_start): nothing of that window ran, and every later launch of the call
// exited at once.  Resume the call where it stopped (the stream is drained):
// the next window epoch (the aborted one's handshake words keep their
// verdict), status RUNNING with the call's forced pivot, and the rest of the
// call on the launch-per-phase chain, which needs no co-residency -- or, for a
// peer-only shard, which has no such path, the persistent chain again.
int notres_resume(spx_ctx* ctx, int64_t fc, int64_t fr, int* retries) {
  ctx->chain_reruns++;
  const bool lazy_ok = !ctx->sharded || ctx->comm || ctx->loop;
  // only CONSECUTIVE aborts count (the same pivot aborted again and again): a
  // long solve with sporadic aborts, each rerun successfully, never gives up
  // (ctx->h_st is current: every caller pulled the State first)
  const auto now = std::chrono::steady_clock::now();
  if (ctx->h_st->iters != ctx->notres_at || *retries == 0) {
    *retries = 0;
    ctx->notres_since = now;
  }
  ctx->notres_at = ctx->h_st->iters;
  // (round 6, VERDICT r5 do-this 4: a late-draining peer used to make its
  // peers give up after 16 consecutive aborts, ~1.7 s; now they keep
  // rerunning for peer_rerun_s, SPX_PEER_RERUN_S, default 30 s)
  if (!lazy_ok && ++*retries > NOTRES_RETRIES &&
      std::chrono::duration<double>(now - ctx->notres_since).count() > ctx->peer_rerun_s) {
    ctx->err = "persistent chain: blocks not co-resident after repeated reruns for " +
               std::to_string(ctx->peer_rerun_s) +
               " s (peer-only shard: no launch-per-phase path; a peer never drained?)";
    return SPX_E_STATE;
  }
  uint32_t e = 0;
  HIPC(hipMemcpyAsync(&e, ctx->wins[0].epoch, sizeof(e), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  e = (e + 1u) & TAG_EPOCH;
  HIPC(hipMemcpyAsync(ctx->wins[0].epoch, &e, sizeof(e), hipMemcpyHostToDevice, ctx->stream));
  if (lazy_ok && !ctx->chain_denied) {
    ctx->chain_denied = true;
    drop_graphs(ctx);
  }
  return set_state_fields(ctx, ST_RUNNING, fc, fr);
}

// An spx_run_pivots request does not wait for its launches, so it cannot
// rerun a window whose persistent chain aborted at its start handshake
// (ST_NOTRES: that window and the rest of the request did nothing).  The
// points that drain the stream (spx_sync, spx_state, the getters, the next
// call) finish it instead: the missing pivots run with the launch-per-phase
// chain (a peer-only shard: the persistent chain again), as spx_solve's own
// rerun does, so the request ends where it would have.
int rp_recover(spx_ctx* ctx) {
  // (every reader of the tableau comes through here: no leaving-row fix of a
  // fold window may still be owed, whatever call left it)
  if (const int rc = settle_fold(ctx)) return rc;
  if (ctx->rp_target < 0) return SPX_OK;
  const int64_t target = ctx->rp_target;
  ctx->rp_target = -1;
  int retries = 0;
  for (;;) {
    HIPC(hipMemcpyAsync(ctx->h_st, ctx->st, sizeof(State), hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    if (ctx->h_st->status != ST_NOTRES || ctx->h_st->iters >= target) {
      ctx->st_fresh = true;
      return SPX_OK;
    }
    ctx->st_fresh = false;
    int rc = notres_resume(ctx, -1, -1, &retries);
    for (int64_t left = target - ctx->h_st->iters; !rc && left > 0;) {
      const int n = (int)std::min<int64_t>(left, 1 << 20);
      rc = enqueue_pivots(ctx, n, 0);
      left -= n;
    }
    if (!rc) rc = settle_fold(ctx);
    if (rc) return rc;
  }
}

int alloc_common(spx_ctx* ctx, int64_t m_local, int64_t N, int64_t m_global, int64_t row0) {
  const int pad = ctx->ld_pad >= 0 ? ctx->ld_pad : (m_local >= 4096 ? 256 : 0);
  const int64_t ld = std::max<int64_t>(64, round_up(m_local, 64)) + pad;
  // A single-GPU reload of the loaded shape keeps every buffer and only clears
  // them again (round 6: the reference's user path solves small LPs one after
  // another on a pooled context, and ~30 hipMalloc / hipFree pairs were most
  // of a 0.5 ms load; tests/test_gpu_user_path.py).  Row shards always take
  // the allocation path below (their exported buffers go through the pool).
  bool reuse = !ctx->sharded && !ctx->loop && ctx->A && ctx->m_local == m_local &&
               ctx->N == N && ctx->m_global == m_global && ctx->row0 == row0 && ctx->ld == ld;
  if (reuse) {
    choose_geometry(ctx);  // (knobs set since the last load may move the partial counts)
    reuse = enter_part_len(ctx) <= ctx->epl_alloc && ratio_part_len(ctx) <= ctx->rpl_alloc;
  }
  HIPC(hipSetDevice(ctx->device));
  // shards: every rank's records, two parity halves and the window-end plane
  // (peers write them over xGMI: uncached, so this GPU's L2 never serves a
  // stale copy to the local polls; plain memory between virtual ranks)
  // (+2 planes: the start handshake's arrivals and verdict word; shards also
  // the IPC release plane and the owner-push inbox, spx_chain.hpp)
  const size_t gq = sizeof(unsigned long long) *
                    (ctx->sharded ? (size_t)shard_record_granules(N)
                                  : (size_t)(HS_PLANE_1GPU + 2) * CHAIN_MAX_BLOCKS);
  if (reuse) {
    // The captured graphs stay too: their launches name the same buffers and
    // sizes, everything a call changes is read from device memory (Params /
    // State, written by call_begin_kernel), and every knob that changes a
    // launch drops them in its setter.  (A small LP's spx_solve spent ~0.4 ms
    // capturing its 32-pivot graph after every reload.)
    ctx->loaded = false;
  } else {
    free_buffers(ctx);
    ctx->m_local = m_local;
    ctx->m_global = m_global;
    ctx->row0 = row0;
    ctx->N = N;
    ctx->ld = ld;
    choose_geometry(ctx);
    ctx->hist_cap = 1 << 20;
    ctx->A_bytes = sizeof(double) * ctx->ld * N;
    // (the buffers a row shard may export come from its pool, spx_ctx::pool)
    const bool exportable = ctx->sharded && !ctx->loop;
    if (exportable) {
      if (const int rc = pool_take(ctx, POOL_TABLEAU, ctx->A_bytes, false,
                                   reinterpret_cast<void**>(&ctx->A), &ctx->A_bytes))
        return rc;
    } else {
      HIPC(hipMalloc(&ctx->A, ctx->A_bytes));
    }
    HIPC(hipMalloc(&ctx->obj, sizeof(double) * N));
    HIPC(hipMalloc(&ctx->F, sizeof(double) * 2 * ctx->ld));
    HIPC(hipMalloc(&ctx->P, sizeof(double) * N));
    HIPC(hipMalloc(&ctx->list, sizeof(int) * N));
    HIPC(hipMalloc(&ctx->basis, sizeof(int64_t) * std::max<int64_t>(1, m_global)));
    HIPC(hipMalloc(&ctx->hist, sizeof(int64_t) * 2 * ctx->hist_cap));
    ctx->epl_alloc = enter_part_len(ctx);
    ctx->rpl_alloc = ratio_part_len(ctx);
    HIPC(hipMalloc(&ctx->enter_part, sizeof(Key) * ctx->epl_alloc));  // per wave / chain block
    HIPC(hipMalloc(&ctx->ratio_part, sizeof(Key) * ctx->rpl_alloc));
    // shared by both window sets: column tags, the window epoch, the fold words
    HIPC(hipMalloc(&ctx->wins[0].tag, sizeof(uint32_t) * N));
    HIPC(hipMalloc(&ctx->wins[0].epoch, sizeof(uint32_t)));
    HIPC(hipMalloc(&ctx->wins[0].fix, sizeof(int32_t) * 8));
    for (int x = 0; x < 2; ++x) {
      Window& w = ctx->wins[x];
      w.tag = ctx->wins[0].tag;
      w.epoch = ctx->wins[0].epoch;
      w.fix = ctx->wins[0].fix;
      w.sid = x;
      HIPC(hipMalloc(&w.F, sizeof(double) * KW * ctx->ld));
      HIPC(hipMalloc(&w.P, sizeof(double) * KW * N));
      HIPC(hipMalloc(&w.r, sizeof(int64_t) * KW));
      HIPC(hipMalloc(&w.c, sizeof(int64_t) * KW));
      HIPC(hipMalloc(&w.made, sizeof(int32_t) * KW));
      HIPC(hipMalloc(&w.nlist, sizeof(int32_t)));
      HIPC(hipMalloc(&w.rec, sizeof(double) * RECW * N));
      HIPC(hipMalloc(&w.frt, sizeof(double) * KW * KW));
      HIPC(hipMalloc(&w.Pf, sizeof(double) * KW * N));
    }
    HIPC(hipMalloc(&ctx->gr_enter, sizeof(unsigned long long) * ENTER_REC * CHAIN_MAX_BLOCKS));
    ctx->gr_bytes = gq;
    if (exportable) {
      if (const int rc = pool_take(ctx, POOL_RECORDS, gq, true,
                                   reinterpret_cast<void**>(&ctx->gr_ratio), &ctx->gr_bytes))
        return rc;
    } else {
      HIPC(hipMalloc(&ctx->gr_ratio, gq));
    }
    if (ctx->sharded) {
      ctx->gstride = round_up(PAYLOAD_HDR + (int64_t)sizeof(double) * N, 256);
      HIPC(hipMalloc(&ctx->sendbuf, ctx->gstride));
      HIPC(hipMalloc(&ctx->recvbuf, ctx->gstride * ctx->nranks));
    }
  }
  // every load starts from zeroed buffers, reused or new: the tableau by a
  // fill, the rest in one launch (zero_spans_kernel)
  ZeroSpans z{};
  uint64_t most = 0;
  auto span = [&](void* ptr, size_t bytes) {
    z.p[z.n] = static_cast<uint32_t*>(ptr);
    z.words[z.n] = bytes / 4;  // (every size here is a multiple of 4 B)
    most = std::max<uint64_t>(most, bytes / 16);
    ++z.n;
  };
  span(ctx->wins[0].tag, sizeof(uint32_t) * N);
  span(ctx->wins[0].epoch, sizeof(uint32_t));
  span(ctx->wins[0].fix, sizeof(int32_t) * 8);
  for (int x = 0; x < 2; ++x) {
    Window& w = ctx->wins[x];
    span(w.Pf, sizeof(double) * KW * N);
    span(w.frt, sizeof(double) * KW * KW);
    span(w.nlist, sizeof(int32_t));
    span(w.rec, sizeof(double) * RECW * N);
    span(w.F, sizeof(double) * KW * ctx->ld);
    span(w.P, sizeof(double) * KW * N);
    span(w.made, sizeof(int32_t) * KW);
    span(w.r, sizeof(int64_t) * KW);
    span(w.c, sizeof(int64_t) * KW);
  }
  ctx->wpar = 0;
  ctx->last_fold = false;
  span(ctx->gr_enter, sizeof(unsigned long long) * ENTER_REC * CHAIN_MAX_BLOCKS);
  span(ctx->gr_ratio, gq);
  if (ctx->sharded) span(ctx->sendbuf, ctx->gstride);
  span(ctx->F, sizeof(double) * 2 * ctx->ld);
  span(ctx->P, sizeof(double) * N);
  static_assert(3 + 2 * 9 + 5 <= ZERO_SPANS_MAX, "zero spans");
  const unsigned gx = (unsigned)std::min<uint64_t>(1024, std::max<uint64_t>(1, (most + BLK - 1) / BLK));
  hipLaunchKernelGGL(zero_spans_kernel, dim3(gx, (unsigned)z.n), dim3(BLK), 0, ctx->stream, z);
  HIPC(hipGetLastError());
  HIPC(hipMemsetAsync(ctx->A, 0, sizeof(double) * ctx->ld * N, ctx->stream));
  std::memset(ctx->h_st, 0, sizeof(State));
  ctx->h_st->status = ST_RUNNING;
  ctx->h_st->forced_c = -1;
  ctx->h_st->forced_r = -1;
  ctx->h_st->hist_cap = ctx->hist_cap;
  HIPC(hipMemcpyAsync(ctx->st, ctx->h_st, sizeof(State), hipMemcpyHostToDevice, ctx->stream));
  ctx->st_fresh = false;  // (the load's first call pulls once)
  return SPX_OK;
}

}  // namespace

extern "C" {

void spx_default_opts(spx_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->rule = SPX_RULE_DANTZIG;
  o->skip_zero_cols = 1;
  o->eps_opt = 1e-9;
  o->eps_piv = 1e-12;
  o->max_iters = 0;
  o->time_limit_s = 0.0;
  o->n_enter = 0;
  o->chunk = 32;
  o->use_graph = 1;
}

int spx_abi_version(void) { return SPX_ABI_VERSION; }

const char* spx_last_error(const spx_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int spx_create(spx_ctx** out, int device) {
  if (!out) return SPX_E_ARG;
  *out = nullptr;
  spx_ctx* ctx = new spx_ctx();
  ctx->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&ctx->prm, sizeof(Params));
  if (e == hipSuccess) e = hipMalloc(&ctx->st, sizeof(State));
  if (e == hipSuccess) e = hipHostMalloc(&ctx->h_st, sizeof(State), hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc(&ctx->h_poll, 2 * sizeof(State), hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc(&ctx->h_stop, sizeof(int32_t), hipHostMallocMapped);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&ctx->d_stop, ctx->h_stop, 0);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_poll[0], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_poll[1], hipEventDisableTiming);
  if (e != hipSuccess) {
    ctx->err = std::string("spx_create: ") + hipGetErrorString(e);
    *out = ctx;  // caller may read the error, then destroy
    return SPX_E_HIP;
  }
  std::memset(ctx->h_st, 0, sizeof(State));
  *ctx->h_stop = 0;
  // tuning hook: SPX_FLUSH_TAIL=x (0..50) overrides the flush's tail share
  if (const char* ft = std::getenv("SPX_FLUSH_TAIL"))
    ctx->flush_tail = std::max(0, std::min(50, std::atoi(ft)));
  // windows per replayed graph (1..16; tuning hook)
  if (const char* gw = std::getenv("SPX_GRAPH_WINDOWS"))
    ctx->graph_windows = std::max(1, std::min(16, std::atoi(gw)));
  if (const char* f = std::getenv("SPX_PEER_RERUN_S"))
    ctx->peer_rerun_s = std::max(0.0, std::atof(f));
  // the row_fix fold (A/B hook): SPX_ROW_FIX_FOLD=1 on
  if (const char* f = std::getenv("SPX_ROW_FIX_FOLD")) ctx->fold = std::atoi(f) != 0;
  *out = ctx;
  return SPX_OK;
}

int spx_comm_unique_id(char out_id[128]) {
  if (!out_id) return SPX_E_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return SPX_E_RCCL;
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  std::memcpy(out_id, &id, sizeof(id));
  return SPX_OK;
}

int spx_create_sharded(spx_ctx** out, int device, int rank, int nranks, const char id[128]) {
  int rc = spx_create(out, device);
  if (rc) return rc;
  spx_ctx* ctx = *out;
  CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks && id, "bad rank/nranks/id");
  ctx->rank = rank;
  ctx->nranks = nranks;
  ctx->sharded = true;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  NCCLC(ncclCommInitRank(&ctx->comm, nranks, uid, rank));
  return SPX_OK;
}

static std::mutex g_loop_mu;  // guards the registry of in-process groups only
static std::map<std::string, LoopGroup*> g_loops;

int spx_create_sharded_local(spx_ctx** out, int device, int rank, int nranks,
                             const char id[128]) {
  int rc = spx_create(out, device);
  if (rc) return rc;
  spx_ctx* ctx = *out;
  CHECK_ARG(nranks >= 1 && nranks <= LOOP_MAX && rank >= 0 && rank < nranks && id,
            "bad rank/nranks/id (loopback groups hold at most 16 ranks)");
  ctx->rank = rank;
  ctx->nranks = nranks;
  ctx->sharded = true;
  HIPC(hipEventCreateWithFlags(&ctx->ev_ready, hipEventDisableTiming));
  HIPC(hipEventCreateWithFlags(&ctx->ev_done, hipEventDisableTiming));
  std::lock_guard<std::mutex> lk(g_loop_mu);
  const std::string key(id, 128);
  LoopGroup*& G = g_loops[key];
  if (!G) {
    G = new LoopGroup();
    G->n = nranks;
    G->key = key;
    G->members.assign(nranks, nullptr);
  }
  if (G->n != nranks || G->members[rank] != nullptr) {
    ctx->err = "loopback group: rank taken or size mismatch";
    return SPX_E_ARG;
  }
  G->members[rank] = ctx;
  G->refs++;
  ctx->loop = G;
  return SPX_OK;
}

int spx_create_sharded_peer(spx_ctx** out, int device, int rank, int nranks) {
  int rc = spx_create(out, device);
  if (rc) return rc;
  spx_ctx* ctx = *out;
  CHECK_ARG(nranks >= 1 && nranks <= CHAIN_MAX_RANKS && rank >= 0 && rank < nranks,
            "bad rank/nranks (peer shards: at most 16 ranks)");
  ctx->rank = rank;
  ctx->nranks = nranks;
  ctx->sharded = true;
  return SPX_OK;
}

// ---- the row-sharded persistent chain's peers ---------------
namespace {
struct PeerBlob {
  uint32_t magic;
  int32_t rank, nranks, device;
  hipIpcMemHandle_t hA, hR;  // this rank's tableau and ratio-record buffer
  int64_t ld, row0, m_local, N, m_global;
  char bus[64];              // PCI bus id: which ranks share a GPU
  int32_t n_cu, chain_mode, chain_min_blocks, push;  // what the shard geometry depends on
  int32_t no_export, pad;    // this rank's load is not exported (a full pool): no peer chain
};
constexpr uint32_t PEER_MAGIC = 0x53505853u;  // "SPXS" (round 6: + no_export)

// What one rank contributes to the shard chain's geometry (its blob, or a
// virtual rank's context): every rank computes the geometry from ALL ranks'
// inputs, in rank order, so every rank reaches the same decision.
struct ShardIn {
  std::string dev;  // device key (PCI bus id): the ranks sharing a GPU form a group
  int n_cu = 0, mode = 0, min_blocks = 0, push = 0;
  int64_t m_local = 0;
};

// Device groups (ranks sharing a GPU: one start handshake each, their chains
// resident together) and the grid of the row-sharded chain.  B = 0 when the
// grid does not fit: every rank's records in one poll (nranks * B <= 512) and
// each group's blocks on its GPU's CUs.  Rows per block come from the LARGEST
// row block (an uneven split may give a rank more rows than the even share:
// every row must be owned by one thread of its block).
int shard_geometry(spx_ctx* ctx, ChainPeers& pe, const std::vector<ShardIn>& in, int* B_out,
                   int* cb_out) {
  const int nr = pe.nranks;
  for (int q = 1; q < nr; ++q) {
    CHECK_ARG(in[q].mode == in[0].mode && in[q].min_blocks == in[0].min_blocks,
              "peer chain: ranks disagree on the chain mode (spx_set_chain)");
    CHECK_ARG(in[q].push == in[0].push,
              "peer chain: ranks disagree on the leaving-row transport (spx_set_peer_push)");
  }
  pe.push = in[0].push;
  pe.ngroups = 0;
  int gof[CHAIN_MAX_RANKS];
  for (int q = 0; q < nr; ++q) {
    int g = -1;
    for (int h = 0; h < pe.ngroups && g < 0; ++h)
      if (in[pe.gleader[h]].dev == in[q].dev) g = h;
    if (g < 0) {
      g = pe.ngroups++;
      pe.gleader[g] = q;
      pe.gmask[g] = 0u;
    }
    pe.gmask[g] |= 1u << q;
    gof[q] = g;
  }
  pe.group = gof[pe.rank];
  int64_t rows = 0;
  int cu_min = CHAIN_MAX_BLOCKS;
  for (const ShardIn& x : in) {
    rows = std::max(rows, x.m_local);
    cu_min = std::min(cu_min, x.n_cu > 0 ? x.n_cu : 256);
  }
  const int cb = chain_cb(in[0].mode, std::max<int64_t>(ctx->N, rows), cu_min);
  const int64_t need = chain_need(ctx->N, rows, cb, in[0].min_blocks);
  bool ok = in[0].mode != 1 && need * nr <= CHAIN_SH_SLOTS;
  for (int g = 0; g < pe.ngroups; ++g) {
    int cap = CHAIN_MAX_BLOCKS;
    for (int q = 0; q < nr; ++q)
      if ((pe.gmask[g] >> q) & 1u) cap = std::min(cap, in[q].n_cu > 0 ? in[q].n_cu : 256);
    ok = ok && need * __builtin_popcount(pe.gmask[g]) <= cap;
  }
  *B_out = ok ? (int)need : 0;
  *cb_out = cb;
  return SPX_OK;
}

// Install a peers table: host copy, device copy (with this rank's stop word), on.
int peer_commit(spx_ctx* ctx, const ChainPeers& pe, int B, int cb) {
  ctx->peers = pe;
  ctx->peers.stop_req = (const int32_t*)ctx->d_stop;
  if (!ctx->d_peers) HIPC(hipMalloc(&ctx->d_peers, sizeof(ChainPeers)));
  HIPC(hipMemcpyAsync(ctx->d_peers, &ctx->peers, sizeof(ChainPeers), hipMemcpyHostToDevice,
                      ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  ctx->peer_same_dev = __builtin_popcount(pe.gmask[pe.group]);
  ctx->peer_B = B;
  ctx->peer_cb = cb;
  ctx->peer_ok = true;
  drop_graphs(ctx);
  return SPX_OK;
}

int peer_check(spx_ctx* ctx) {
  CHECK_ARG(ctx->sharded && ctx->loaded, "peer chain: a loaded sharded context is needed");
  CHECK_ARG(ctx->nranks <= CHAIN_MAX_RANKS, "peer chain: at most 16 ranks");
  return SPX_OK;
}
}  // namespace

int spx_peer_blob_size(void) { return (int)sizeof(PeerBlob); }

// This rank's exchange blob (IPC handles of its tableau and record buffer,
// its rows and GPU), to be all-gathered by the caller and given to
// spx_peer_import on every rank.  Valid until the next load.
int spx_peer_export(spx_ctx* ctx, void* out, int64_t cap) {
  if (!ctx) return SPX_E_ARG;
  int rc = peer_check(ctx);
  if (rc) return rc;
  CHECK_ARG(out && cap >= (int64_t)sizeof(PeerBlob), "blob buffer too small");
  PeerBlob b;
  std::memset(&b, 0, sizeof(b));
  b.magic = PEER_MAGIC;
  b.rank = ctx->rank;
  b.nranks = ctx->nranks;
  b.device = ctx->device;
  HIPC(hipSetDevice(ctx->device));
  b.no_export = ctx->export_blocked ? 1 : 0;
  if (!ctx->export_blocked) {
    HIPC(hipIpcGetMemHandle(&b.hA, ctx->A));
    HIPC(hipIpcGetMemHandle(&b.hR, ctx->gr_ratio));
    ctx->ever_exported.insert(ctx->A);
    ctx->ever_exported.insert(ctx->gr_ratio);
  }
  b.ld = ctx->ld;
  b.row0 = ctx->row0;
  b.m_local = ctx->m_local;
  b.N = ctx->N;
  b.m_global = ctx->m_global;
  HIPC(hipDeviceGetPCIBusId(b.bus, (int)sizeof(b.bus) - 1, ctx->device));
  // test hook (round 6): SPX_PEER_GROUP_TAG=x makes this rank's device key
  // "<bus id>#x", so ranks on ONE GPU with different tags form different
  // device groups -- each its own start handshake, then the cross-group
  // verdict wait that ranks on different GPUs run (chain_start), which one
  // GPU can then execute.  The caller keeps all groups' blocks within the CUs.
  if (const char* tag = std::getenv("SPX_PEER_GROUP_TAG")) {
    const size_t n = strnlen(b.bus, sizeof(b.bus));
    std::snprintf(b.bus + n, sizeof(b.bus) - n, "#%s", tag);
  }
  if (!ctx->n_cu) ctx->n_cu = device_cus(ctx->device);
  b.n_cu = ctx->n_cu;
  b.chain_mode = ctx->chain_mode;
  b.chain_min_blocks = ctx->chain_min_blocks;
  b.push = ctx->peer_push;
  std::memcpy(out, &b, sizeof(b));
  return SPX_OK;
}

// Map every peer's tableau and record buffer (blobs: nranks blobs in rank
// order, spx_peer_blob_size() bytes each).  Collective in effect: every rank
// imports after every rank exported; afterwards windows of this context run
// the row-sharded persistent chain when its grid fits.
int spx_peer_import(spx_ctx* ctx, const void* blobs, int nranks) {
  if (!ctx) return SPX_E_ARG;
  int rc = peer_check(ctx);
  if (rc) return rc;
  CHECK_ARG(blobs && nranks == ctx->nranks, "peer import: one blob per rank");
  close_peers(ctx);
  HIPC(hipSetDevice(ctx->device));
  const PeerBlob* bl = static_cast<const PeerBlob*>(blobs);
  ChainPeers pe{};
  pe.rank = ctx->rank;
  pe.nranks = nranks;
  std::vector<ShardIn> in(nranks);
  int64_t rows_sum = 0;
  for (int q = 0; q < nranks; ++q) {
    const PeerBlob& b = bl[q];
    CHECK_ARG(b.magic == PEER_MAGIC && b.rank == q && b.nranks == nranks && b.N == ctx->N &&
                  b.m_global == ctx->m_global && b.m_local >= 0,
              "peer import: blob mismatch (rank order, shape, library version)");
    CHECK_ARG(b.row0 == rows_sum, "peer import: the ranks' row blocks must tile 0..m in rank order");
    rows_sum += b.m_local;
    in[q].dev = std::string(b.bus, strnlen(b.bus, sizeof(b.bus)));
    in[q].n_cu = b.n_cu;
    in[q].mode = b.chain_mode;
    in[q].min_blocks = b.chain_min_blocks;
    in[q].push = b.push;
    in[q].m_local = b.m_local;
  }
  CHECK_ARG(rows_sum == ctx->m_global, "peer import: the row blocks do not cover every row");
  for (int q = 0; q < nranks; ++q)
    if (bl[q].no_export) {  // (every rank sees the same blobs: every rank returns this)
      ctx->err = "peer chain unavailable for this load: rank " + std::to_string(q) +
                 "'s pool of exported buffers is full (4 sizes per role, DESIGN.md 5c); its "
                 "windows run the RCCL path where a communicator exists";
      return SPX_E_NOPEER;
    }
  int B = 0, cb = BLK;
  if ((rc = shard_geometry(ctx, pe, in, &B, &cb))) return rc;
  for (int q = 0; q < nranks; ++q) {
    const PeerBlob& b = bl[q];
    pe.ld[q] = b.ld;
    pe.row0[q] = b.row0;
    if (q == ctx->rank) {
      pe.A[q] = ctx->A;
      pe.ratio[q] = ctx->gr_ratio;
      continue;
    }
    void* pa = nullptr;
    void* pr = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&pa, b.hA, hipIpcMemLazyEnablePeerAccess);
    if (e == hipSuccess) ctx->ipc_open.push_back(pa);
    if (e == hipSuccess) e = hipIpcOpenMemHandle(&pr, b.hR, hipIpcMemLazyEnablePeerAccess);
    if (e == hipSuccess) ctx->ipc_open.push_back(pr);
    if (e != hipSuccess) {
      close_peers(ctx);
      ctx->err = std::string("peer import: hipIpcOpenMemHandle: ") + hipGetErrorString(e);
      return SPX_E_HIP;
    }
    pe.A[q] = static_cast<const double*>(pa);
    pe.ratio[q] = static_cast<unsigned long long*>(pr);
  }
  if ((rc = peer_commit(ctx, pe, B, cb))) return rc;
  ctx->peer_gen++;  // (every rank imports together: the same generation everywhere)
  ctx->imported_load = true;
  return SPX_OK;
}

// Virtual ranks (spx_create_sharded_local): the peers are this process's
// group members.  Every rank calls it after its load (it meets the others).
int spx_peer_chain_local(spx_ctx* ctx) {
  if (!ctx) return SPX_E_ARG;
  int rc = peer_check(ctx);
  if (rc) return rc;
  CHECK_ARG(ctx->loop != nullptr, "spx_peer_chain_local: not a virtual-rank context");
  LoopGroup* G = ctx->loop;
  if (!G->barrier()) return loop_fail(ctx);  // every member loaded
  ChainPeers pe{};
  pe.rank = ctx->rank;
  pe.nranks = ctx->nranks;
  std::vector<ShardIn> in(G->n);
  int64_t rows_sum = 0;
  // (every rank checks the same members in the same order, so all return the
  // same error before the second barrier, or none does)
  for (int q = 0; q < G->n; ++q) {
    spx_ctx* m = G->members[q];
    CHECK_ARG(m && m->loaded && m->N == ctx->N && m->m_global == ctx->m_global,
              "spx_peer_chain_local: group member not loaded / shape mismatch");
    // the chain dereferences the members' tableaux and record buffers as
    // plain device pointers: no peer mapping between GPUs here
    CHECK_ARG(m->device == G->members[0]->device,
              "spx_peer_chain_local: virtual ranks of a peer chain must share one GPU "
              "(use one process per GPU and spx_peer_export / spx_peer_import)");
    CHECK_ARG(m->row0 == rows_sum, "spx_peer_chain_local: row blocks must tile 0..m in rank order");
    rows_sum += m->m_local;
    pe.A[q] = m->A;
    pe.ratio[q] = m->gr_ratio;
    pe.ld[q] = m->ld;
    pe.row0[q] = m->row0;
    in[q].dev = std::to_string(m->device);
    in[q].n_cu = device_cus(m->device);
    in[q].mode = m->chain_mode;
    in[q].min_blocks = m->chain_min_blocks;
    in[q].push = m->peer_push;
    in[q].m_local = m->m_local;
  }
  CHECK_ARG(rows_sum == ctx->m_global, "spx_peer_chain_local: row blocks do not cover every row");
  int B = 0, cb = BLK;
  if ((rc = shard_geometry(ctx, pe, in, &B, &cb))) return rc;
  if (!G->barrier()) return loop_fail(ctx);  // nobody reloads while the others read
  close_peers(ctx);
  return peer_commit(ctx, pe, B, cb);
}

int spx_destroy(spx_ctx* ctx) {
  if (!ctx) return SPX_OK;
  if (ctx->loop) {
    std::lock_guard<std::mutex> lk(g_loop_mu);
    LoopGroup* G = ctx->loop;
    G->members[ctx->rank] = nullptr;
    if (--G->refs == 0) {
      g_loops.erase(G->key);
      delete G;
    }
    ctx->loop = nullptr;
  }
  if (ctx->ev_ready) (void)hipEventDestroy(ctx->ev_ready);
  if (ctx->ev_done) (void)hipEventDestroy(ctx->ev_done);
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  {
    ChainAdmission& a = adm();
    std::lock_guard<std::mutex> lk(a.mu);
    adm_settle_locked(a, ctx, true);
    a.deferred.erase(ctx);
    while (ctx->adm_calls > 0) adm_release_locked(a, ctx);  // (error paths)
  }
  if (ctx->adm_ev) (void)hipEventDestroy(ctx->adm_ev);
  // the peers' release marks (close_peers) for every record buffer this
  // context exported that peers imported -- the current one if this load was
  // imported, and each pooled one under the generation it was imported with
  // (a reload without a re-import has no marks to wait for in the
  // current buffer) -- within one bounded wait, then every buffer goes
  free_buffers(ctx);  // (closes this context's mappings of its peers; the
                      // current exported buffers join the pool, with their generation)
  {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(10);
    for (const auto& e : ctx->pool)
      if (e.role == POOL_RECORDS && e.gen > 0)
        (void)wait_peer_release(ctx, static_cast<const unsigned long long*>(e.p), e.gen, deadline);
  }
  for (const auto& e : ctx->pool) (void)hipFree(e.p);
  ctx->pool.clear();
  ctx->ever_exported.clear();
  for (auto* pool : {&ctx->ev, &ctx->evc})
    for (auto& e : *pool) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  dfree(ctx->prm);
  dfree(ctx->st);
  if (ctx->h_st) (void)hipHostFree(ctx->h_st);
  if (ctx->h_poll) (void)hipHostFree(ctx->h_poll);
  if (ctx->h_stop) (void)hipHostFree(ctx->h_stop);
  dfree(ctx->d_peers);
  dfree(ctx->stage);
  for (hipEvent_t ev : ctx->ev_poll)
    if (ev) (void)hipEventDestroy(ev);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return SPX_OK;
}

// Row-major host rows <-> the column-major tableau, in chunks of rows through
// a device staging buffer (at most ~64 MB, freed after the call): H2D: a 2-D
// copy of the chunk's rows, then transpose_kernel into A; D2H: the transpose
// into the staging buffer, then a 2-D copy into the host rows (pitch ld).
int transfer_rows(spx_ctx* ctx, double* host, int64_t nrows, int64_t cols, int64_t ld,
                  bool to_device) {
  // (rows per chunk: ~64 MB of staging, at most 65535 tiles of 32 rows -- the
  // grid's y limit)
  const int64_t chunk = std::min<int64_t>(
      65535 * 32, std::max<int64_t>(32, std::min<int64_t>(nrows, ((8 << 20) / cols + 31) / 32 * 32)));
  // a staging buffer of at most STAGE_KEEP bytes stays with the context (the
  // per-step snapshots of a small LP, round 6: a hipMalloc / hipFree pair per
  // snapshot was most of its cost); larger ones are freed after the call
  constexpr size_t STAGE_KEEP = (size_t)8 << 20;
  const size_t need = sizeof(double) * chunk * cols;
  double* stage = nullptr;
  const bool keep = need <= STAGE_KEEP;
  if (keep) {
    if (ctx->stage_bytes < need) {
      dfree(ctx->stage);
      ctx->stage_bytes = 0;
      HIPC(hipMalloc(&ctx->stage, need));
      ctx->stage_bytes = need;
    }
    stage = ctx->stage;
  } else {
    HIPC(hipMalloc(&stage, need));
  }
  int rc = SPX_OK;
  for (int64_t i0 = 0; i0 < nrows && rc == SPX_OK; i0 += chunk) {
    const int64_t R = std::min(chunk, nrows - i0);
    const dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((R + 31) / 32));
    hipError_t e;
    if (to_device) {
      e = hipMemcpy2DAsync(stage, sizeof(double) * cols, host + i0 * ld, sizeof(double) * ld,
                           sizeof(double) * cols, R, hipMemcpyHostToDevice, ctx->stream);
      if (e == hipSuccess) {
        hipLaunchKernelGGL(transpose_kernel<true>, grid, dim3(256), 0, ctx->stream,
                           (const double*)stage, ctx->A + i0, R, cols, cols, ctx->ld);
        e = hipGetLastError();
      }
    } else {
      hipLaunchKernelGGL(transpose_kernel<false>, grid, dim3(256), 0, ctx->stream,
                         (const double*)(ctx->A + i0), stage, R, cols, cols, ctx->ld);
      e = hipGetLastError();
      if (e == hipSuccess)
        e = hipMemcpy2DAsync(host + i0 * ld, sizeof(double) * ld, stage, sizeof(double) * cols,
                             sizeof(double) * cols, R, hipMemcpyDeviceToHost, ctx->stream);
    }
    // (the staging buffer is reused by the next chunk: wait for this one)
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
      ctx->err = std::string("row transfer: ") + hipGetErrorString(e);
      rc = SPX_E_HIP;
    }
  }
  if (!keep) (void)hipFree(stage);
  return rc;
}

int spx_load_rows(spx_ctx* ctx, const double* A, int64_t m_local, int64_t cols, int64_t ld,
                  int layout, const double* obj, const int64_t* basis, int64_t m_global,
                  int64_t row0) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(cols >= 1 && m_local >= 0 && m_global >= m_local && row0 >= 0 &&
                row0 + m_local <= m_global,
            "bad dimensions");
  CHECK_ARG(obj && (m_global == 0 || basis) && (m_local == 0 || A), "null buffer");
  CHECK_ARG(layout == SPX_ROW_MAJOR || layout == SPX_COL_MAJOR, "bad layout");
  CHECK_ARG(m_local == 0 || (layout == SPX_ROW_MAJOR ? ld >= cols : ld >= m_local), "bad ld");
  CHECK_ARG(cols < INT32_MAX, "too many columns");
  int rc = alloc_common(ctx, m_local, cols, m_global, row0);
  if (rc) return rc;
  if (m_local > 0) {
    // (the column padding rows, ld > m_local, hold zeros: alloc_common cleared
    // the ld * N doubles, whatever a pooled buffer held)
    if (layout == SPX_COL_MAJOR) {
      HIPC(hipMemcpy2DAsync(ctx->A, sizeof(double) * ctx->ld, A, sizeof(double) * ld,
                            sizeof(double) * m_local, cols, hipMemcpyHostToDevice,
                            ctx->stream));
    } else {
      // row-major host rows: copied in chunks into a device staging buffer,
      // transposed there into the column-major tableau (the host transpose
      // this replaces ran at ~2 GB/s; tools/pcie_rate.py)
      rc = transfer_rows(ctx, const_cast<double*>(A), m_local, cols, ld, true);
      if (rc) return rc;
    }
  }
  HIPC(hipMemcpyAsync(ctx->obj, obj, sizeof(double) * cols, hipMemcpyHostToDevice, ctx->stream));
  if (m_global > 0)
    HIPC(hipMemcpyAsync(ctx->basis, basis, sizeof(int64_t) * m_global, hipMemcpyHostToDevice,
                        ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  ctx->loaded = true;
  return SPX_OK;
}

int spx_load(spx_ctx* ctx, const double* T, int64_t rows, int64_t cols, int64_t ld, int layout,
             const int64_t* basis) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(T && rows >= 1 && cols >= 1, "bad tableau");
  CHECK_ARG(!ctx->sharded || ctx->nranks == 1, "use spx_load_rows on a sharded context");
  const int64_t m = rows - 1;
  std::vector<double> objrow((size_t)cols);
  for (int64_t j = 0; j < cols; ++j)
    objrow[j] = (layout == SPX_ROW_MAJOR) ? T[m * ld + j] : T[j * ld + m];
  return spx_load_rows(ctx, T, m, cols, ld, layout, objrow.data(), basis, m, 0);
}

int spx_set_objective(spx_ctx* ctx, const double* obj) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(ctx->loaded && obj, "no tableau / null objective");
  HIPC(hipMemcpyAsync(ctx->obj, obj, sizeof(double) * ctx->N, hipMemcpyHostToDevice,
                      ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  return SPX_OK;
}

int spx_get_tableau(spx_ctx* ctx, double* out, int64_t ld, int layout) {
  if (!ctx) return SPX_E_ARG;
  if (int rc = rp_recover(ctx)) return rc;
  CHECK_ARG(ctx->loaded && out, "no tableau / null buffer");
  CHECK_ARG(layout == SPX_ROW_MAJOR || layout == SPX_COL_MAJOR, "bad layout");
  const int64_t rows = ctx->m_local + 1, N = ctx->N;
  CHECK_ARG(layout == SPX_ROW_MAJOR ? ld >= N : ld >= rows, "bad ld");
  const int64_t ml = ctx->m_local;
  if (layout == SPX_ROW_MAJOR) {
    // rows through a device transpose and one 2-D copy per chunk (the host
    // transpose this replaces ran at ~2 GB/s; tools/pcie_rate.py)
    if (ml > 0) {
      const int rc = transfer_rows(ctx, out, ml, N, ld, false);
      if (rc) return rc;
    }
    HIPC(hipMemcpyAsync(out + ml * ld, ctx->obj, sizeof(double) * N, hipMemcpyDeviceToHost,
                        ctx->stream));
  } else {
    if (ml > 0)
      HIPC(hipMemcpy2DAsync(out, sizeof(double) * ld, ctx->A, sizeof(double) * ctx->ld,
                            sizeof(double) * ml, N, hipMemcpyDeviceToHost, ctx->stream));
    // the objective row: one element per column, ld apart
    HIPC(hipMemcpy2DAsync(out + ml, sizeof(double) * ld, ctx->obj, sizeof(double),
                          sizeof(double), N, hipMemcpyDeviceToHost, ctx->stream));
  }
  HIPC(hipStreamSynchronize(ctx->stream));
  return SPX_OK;
}

int spx_get_objective(spx_ctx* ctx, double* out) {
  if (!ctx) return SPX_E_ARG;
  if (int rc = rp_recover(ctx)) return rc;
  CHECK_ARG(ctx->loaded && out, "no tableau / null buffer");
  HIPC(hipMemcpyAsync(out, ctx->obj, sizeof(double) * ctx->N, hipMemcpyDeviceToHost,
                      ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  return SPX_OK;
}

int spx_get_basis(spx_ctx* ctx, int64_t* out) {
  if (!ctx) return SPX_E_ARG;
  if (int rc = rp_recover(ctx)) return rc;
  CHECK_ARG(ctx->loaded && out, "no tableau / null buffer");
  if (ctx->m_global > 0) {
    HIPC(hipMemcpyAsync(out, ctx->basis, sizeof(int64_t) * ctx->m_global, hipMemcpyDeviceToHost,
                        ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
  }
  return SPX_OK;
}

int spx_get_column(spx_ctx* ctx, int64_t j, double* out) {
  if (!ctx) return SPX_E_ARG;
  if (int rc = rp_recover(ctx)) return rc;
  CHECK_ARG(ctx->loaded && out && j >= 0 && j < ctx->N, "bad column");
  if (ctx->m_local > 0) {
    HIPC(hipMemcpyAsync(out, ctx->A + j * ctx->ld, sizeof(double) * ctx->m_local,
                        hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
  }
  return SPX_OK;
}

int spx_get_history(spx_ctx* ctx, int64_t* rc_pairs, int64_t cap, int64_t* n) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(ctx->loaded && n && (cap == 0 || rc_pairs), "bad history args");
  int rc = pull_state(ctx);
  if (rc) return rc;
  const int64_t have = std::min(ctx->h_st->iters, ctx->hist_cap);
  *n = ctx->h_st->iters;
  const int64_t k = std::min(have, cap);
  if (k > 0) {
    HIPC(hipMemcpyAsync(rc_pairs, ctx->hist, sizeof(int64_t) * 2 * k, hipMemcpyDeviceToHost,
                        ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
  }
  return SPX_OK;
}

int spx_dims(const spx_ctx* ctx, int64_t* m_global, int64_t* m_local, int64_t* cols,
             int64_t* row0) {
  if (!ctx) return SPX_E_ARG;
  if (m_global) *m_global = ctx->m_global;
  if (m_local) *m_local = ctx->m_local;
  if (cols) *cols = ctx->N;
  if (row0) *row0 = ctx->row0;
  return SPX_OK;
}

int spx_solve(spx_ctx* ctx, const spx_opts* opts, spx_result* res) {
  if (!ctx) return SPX_E_ARG;
  spx_opts d;
  spx_default_opts(&d);
  const spx_opts* o = opts ? opts : &d;
  const auto t0 = std::chrono::steady_clock::now();
  AdmCall adm_call(ctx);
  int rc = begin_call(ctx, o, &adm_call);
  if (rc) return rc;
  const int64_t it0 = ctx->h_st->iters;
  const int chunk =
      ctx->win_k ? ctx->win_k * ctx->graph_windows : (o->chunk > 0 ? o->chunk : 32);
  const bool use_graph = o->use_graph != 0 && !ctx->loop && !ctx->time_chain;
  if (use_graph && ctx->win_k) {
    rc = build_graphs_all(ctx, chunk);
    if (rc) return rc;
  }
  int status = SPX_RUNNING;
  // Chunk i+1 is enqueued before chunk i's status is read (a pinned State copy
  // per chunk, polled one chunk behind), so the stream never drains while the
  // host looks.  The chunk after the terminating one only runs early-exiting
  // launches: every kernel checks the device status first.  Single pivots
  // ramp up: chunks of 4, 8, 16 pivots launched directly, then the graph of
  // `chunk` (round 6: a textbook LP stops after a few pivots, and two graphs of
  // 32 pivots were ~0.3 ms of early-exiting launches on its user path).
  auto launch_chunk = [&](int64_t i) -> int {
    const int64_t r4 = (int64_t)4 << std::min<int64_t>(i, 24);
    const int ramp = ctx->win_k || r4 >= chunk ? chunk : (int)r4;
    if (use_graph && ramp == chunk) {
      int r = ctx->win_k ? SPX_OK : build_graph(ctx, chunk);  // (cached after the first)
      if (!r) r = launch_graph(ctx, chunk);
      if (r) return r;
    } else {
      const int r = enqueue_pivots(ctx, ramp, 0);
      if (r) return r;
    }
    HIPC(hipMemcpyAsync(ctx->h_poll + (i & 1), ctx->st, sizeof(State), hipMemcpyDeviceToHost,
                        ctx->stream));
    HIPC(hipEventRecord(ctx->ev_poll[i & 1], ctx->stream));
    return SPX_OK;
  };
  int retries = 0;
  if ((rc = launch_chunk(0))) return rc;
  for (int64_t i = 0;; ++i) {
    if ((rc = launch_chunk(i + 1))) return rc;
    HIPC(hipEventSynchronize(ctx->ev_poll[i & 1]));
    if (ctx->h_poll[i & 1].status == ST_NOTRES) {
      // a window's chain was not co-resident: drain (chunk i+1 only exits
      // early), resume, and restart the pipeline with chunk i+1
      if ((rc = pull_state(ctx)) || (rc = notres_resume(ctx, -1, -1, &retries))) return rc;
      if (use_graph && (rc = build_graph(ctx, chunk))) return rc;
      if ((rc = launch_chunk(i + 1))) return rc;
      continue;
    }
    status = map_status(ctx->h_poll[i & 1].status);
    if (status != SPX_RUNNING) break;
    const double el =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (o->time_limit_s > 0 && el >= o->time_limit_s) {
      if (!ctx->sharded) {
        status = SPX_ITER_LIMIT;
        break;
      }
      // a row shard stops where every rank stops: rank 0 asks its device,
      // whose payload carries the request to all ranks before the same pivot
      // (status ST_LIMIT, read at a later poll); the other ranks wait for it
      if (ctx->rank == 0 && ctx->h_stop) __atomic_store_n(ctx->h_stop, 1, __ATOMIC_SEQ_CST);
    }
  }
  if ((rc = settle_fold(ctx))) return rc;  // the last window's leaving rows
  if ((rc = pull_state(ctx))) return rc;  // the final state (after the extra chunk)
  adm_call.drained = true;
  if (status < 0 || is_fault(ctx->h_st->status)) return fault(ctx);
  double z = 0.0;
  HIPC(hipMemcpyAsync(&z, ctx->obj + (ctx->N - 1), sizeof(double), hipMemcpyDeviceToHost,
                      ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  if (res) {
    res->status = status;
    res->pad = 0;
    res->iters = ctx->h_st->iters - it0;
    res->objective = z;
    res->elapsed_s =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return status;
}

int spx_pivot(spx_ctx* ctx, const spx_opts* opts, int64_t* r, int64_t* c) {
  if (!ctx) return SPX_E_ARG;
  AdmCall adm_call(ctx);
  int rc = begin_call(ctx, opts, &adm_call);
  if (rc) return rc;
  const int64_t it0 = ctx->h_st->iters;
  for (int retries = 0;;) {
    if ((rc = enqueue_pivots(ctx, 1, 0)) || (rc = settle_fold(ctx))) return rc;
    if ((rc = pull_state(ctx))) return rc;
    if (ctx->h_st->status != ST_NOTRES) break;
    if ((rc = notres_resume(ctx, -1, -1, &retries))) return rc;
  }
  adm_call.drained = true;
  const int status = map_status(ctx->h_st->status);
  if (status < 0) return fault(ctx);
  if (status == SPX_RUNNING && ctx->h_st->iters == it0 + 1) {
    if (r) *r = ctx->h_st->r;
    if (c) *c = ctx->h_st->c;
    return SPX_RUNNING;
  }
  if (r) *r = -1;
  if (c) *c = -1;
  return status == SPX_RUNNING ? SPX_E_STATE : status;
}

int spx_pivot_at(spx_ctx* ctx, int64_t r, int64_t c) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(ctx->loaded && r >= 0 && r < ctx->m_global && c >= 0 && c < ctx->N - 1,
            "pivot position out of range");
  AdmCall adm_call(ctx);
  int rc = begin_call(ctx, nullptr, &adm_call, c, r);
  if (rc) return rc;
  // (pull the post-pivot state before writing the forced fields back)
  for (int retries = 0;;) {
    if ((rc = enqueue_pivots(ctx, 1, 0)) || (rc = settle_fold(ctx))) return rc;
    if ((rc = pull_state(ctx))) return rc;
    if (ctx->h_st->status != ST_NOTRES) break;
    if ((rc = notres_resume(ctx, c, r, &retries))) return rc;
  }
  adm_call.drained = true;
  const int32_t st_after = ctx->h_st->status;
  if (is_fault(st_after)) return fault(ctx);
  if ((rc = set_state_fields(ctx, st_after, -1, -1))) return rc;
  if ((rc = pull_state(ctx))) return rc;
  return st_after == ST_RUNNING ? SPX_OK : SPX_E_STATE;
}

int spx_run_pivots(spx_ctx* ctx, const spx_opts* opts, int64_t npivots, int time_elim) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(npivots >= 0 && time_elim >= 0, "npivots / time_elim < 0");
  spx_opts d;
  spx_default_opts(&d);
  const spx_opts* o = opts ? opts : &d;
  AdmCall adm_call(ctx);  // released behind this call's launches (it does not sync)
  int rc = begin_call(ctx, o, &adm_call);
  if (rc) return rc;
  ctx->rp_target = ctx->h_st->iters + npivots;  // (begin_call drained: iters is current)
  // (chain timing records one event pair per window: direct launches, since a
  // replayed graph re-records the same captured events)
  const bool graph = o->use_graph && !ctx->loop && !ctx->time_chain;
  const int unit = ctx->win_k ? ctx->win_k : 1;  // pivots per enqueue unit
  // the whole request as a sequence of units: full windows, then a remainder
  auto enqueue_all = [&](int tk) -> int {
    int64_t done = 0;
    while (done < npivots) {
      const int n = (int)std::min<int64_t>(ctx->win_k ? unit : 1, npivots - done);
      const int r = enqueue_pivots(ctx, n, tk, done);
      if (r) return r;
      done += n;
    }
    return SPX_OK;
  };
  if (time_elim) {
    // Timed: every time_elim-th window (or elimination) is launched directly
    // between two stream events; the untimed windows replay graphs (below).
    // (One graph of the whole request ran 18 % slower at config 3: a hipGraph
    // of ~550 nodes is submitted in batches the GPU overtakes.)
    if (!ctx->win_k || !graph) {
      rc = enqueue_all(time_elim);
      return rc ? rc : settle_fold(ctx);
    }
    // the untimed windows between two timed ones replay the graph of
    // graph_windows windows (the ones an untimed call builds, for every
    // window state, so no graph is captured inside a timed region); shorter
    // runs are launched directly
    const int run = ctx->graph_windows;
    if (time_elim > run && (rc = build_graphs_all(ctx, run * ctx->win_k))) return rc;
    int64_t done = 0;
    for (int64_t w = 0; done < npivots;) {
      const int n = (int)std::min<int64_t>(ctx->win_k, npivots - done);
      const bool timed = w % time_elim == 0;
      if (!timed && time_elim > run && npivots - done >= (int64_t)run * ctx->win_k &&
          (w % time_elim) + run <= time_elim) {
        if ((rc = launch_graph(ctx, run * ctx->win_k))) return rc;
        done += (int64_t)run * ctx->win_k;
        w += run;
        continue;
      }
      if ((rc = enqueue_window(ctx, n, timed))) return rc;
      done += n;
      ++w;
    }
    return settle_fold(ctx);
  }
  if (!time_elim && graph) {
    const int chunk =
        ctx->win_k ? ctx->win_k * ctx->graph_windows : (o->chunk > 0 ? o->chunk : 32);
    if ((rc = build_graphs_all(ctx, chunk))) return rc;
    int64_t left = npivots;
    for (; left >= chunk; left -= chunk)
      if ((rc = launch_graph(ctx, chunk))) return rc;
    if (left > 0 && (rc = enqueue_pivots(ctx, (int)left, 0))) return rc;
    return settle_fold(ctx);
  }
  rc = enqueue_all(time_elim);
  return rc ? rc : settle_fold(ctx);
}

// Windowed (delayed) elimination: K pivots per tableau pass (2..16), 0/1 = off.
#ifdef SPX_PHASE_TIMING
// diagnostic build only: per-wave flush exit stamps (tools/probe_phases.py)
int spx_probe_read_wave(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(spx::spx_probe_wave),
                             sizeof(unsigned long long) * std::min(n, 2 * 4 * 8192)) ==
                 hipSuccess
             ? 0
             : -1;
}
// diagnostic build only (tools/probe_phases.py): copy the phase timestamps
int spx_probe_read(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(spx::spx_probe_buf),
                             sizeof(unsigned long long) * std::min(n, 1024 + 2 * 8192)) ==
                 hipSuccess
             ? 0 : -1;
}
int spx_probe_read_chain(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(spx::spx_probe_chain),
                             sizeof(unsigned long long) *
                                 std::min(n, 32 * spx::PROBE_CHAIN_EV * 256)) == hipSuccess
             ? 0 : -1;
}
int spx_probe_read_chain_hw(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(spx::spx_probe_chain_hw),
                             sizeof(unsigned long long) * std::min(n, 256)) == hipSuccess
             ? 0 : -1;
}
// flush grid of the last window (diagnostic)
int spx_probe_flush_grid(spx_ctx* ctx, int* rch, int* G) {
  *rch = ctx->last_flush_rch;
  *G = ctx->last_flush_G;
  return 0;
}
#endif

int spx_set_window(spx_ctx* ctx, int K) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(K == 0 || K == 1 || K == 2 || K == 4 || K == 8 || K == 12 || K == 16 || K == 24 || K == 28 ||
                K == 32,
            "window must be 0, 1, 2, 4, 8, 12, 16, 24, 28 or 32");
  if (const int rc = settle_fold(ctx)) return rc;  // (its gated row_fix is of the old K)
  ctx->win_k = K <= 1 ? 0 : K;
  drop_graphs(ctx);
  return SPX_OK;
}

// The row_fix fold: 1 the persistent single-GPU chain
// rewrites the previous window's leaving rows, 0 (default) a row_fix launch
// after every window.  Bit-identical either way; measured no faster (the fix
// moves onto the chain's critical path), so off.  SPX_ROW_FIX_FOLD=1 sets 1 at
// create (A/B runs).
int spx_set_row_fix_fold(spx_ctx* ctx, int on) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(on == 0 || on == 1, "row_fix fold must be 0 or 1");
  if (const int rc = settle_fold(ctx)) return rc;
  ctx->fold = on;
  drop_graphs(ctx);
  return SPX_OK;
}

int spx_sync(spx_ctx* ctx) {
  if (!ctx) return SPX_E_ARG;
  HIPC(hipStreamSynchronize(ctx->stream));
  adm_settle(ctx, true);
  return rp_recover(ctx);
}

int spx_state(spx_ctx* ctx, int32_t* status, int64_t* iters, double* objective) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(ctx->loaded, "no tableau loaded");
  int rc = pull_state(ctx);
  if (rc) return rc;
  if (is_fault(ctx->h_st->status)) return fault(ctx);
  if (status) *status = map_status(ctx->h_st->status);
  if (iters) *iters = ctx->h_st->iters;
  if (objective) {
    HIPC(hipMemcpyAsync(objective, ctx->obj + (ctx->N - 1), sizeof(double),
                        hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
  }
  return SPX_OK;
}

// Pivot-choice timing: when on, every window records HIP events around its
// chain (persistent kernel or lazy kernels).  Diagnostic: the event nodes add
// stream time, so bench.py measures it in a pass after its timed region.
int spx_set_chain_timing(spx_ctx* ctx, int on) {
  if (!ctx) return SPX_E_ARG;
  ctx->time_chain = on != 0;
  drop_graphs(ctx);
  return SPX_OK;
}

int spx_chain_timing(spx_ctx* ctx, double* total_ms, int64_t* count, int reset) {
  if (!ctx) return SPX_E_ARG;
  HIPC(hipStreamSynchronize(ctx->stream));
  double tot = 0.0;
  for (size_t i = 0; i < ctx->evc_used; ++i) {
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ctx->evc[i].first, ctx->evc[i].second));
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (count) *count = (int64_t)ctx->evc_used;
  if (reset) ctx->evc_used = 0;
  return SPX_OK;
}

int spx_elim_timing(spx_ctx* ctx, double* total_ms, int64_t* count, int64_t* touched_cols,
                    int reset) {
  if (!ctx) return SPX_E_ARG;
  HIPC(hipStreamSynchronize(ctx->stream));
  double tot = 0.0;
  for (size_t i = 0; i < ctx->ev_used; ++i) {
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ctx->ev[i].first, ctx->ev[i].second));
    tot += ms;
  }
  int rc = pull_state(ctx);
  if (rc) return rc;
  if (total_ms) *total_ms = tot;
  if (count) *count = (int64_t)ctx->ev_used;
  if (touched_cols) *touched_cols = ctx->h_st->touched_total - ctx->touched_at_reset;
  if (reset) {
    ctx->ev_used = 0;
    ctx->touched_at_reset = ctx->h_st->touched_total;
  }
  return SPX_OK;
}

// Tuning knob: elimination rows per thread R (2/4/8, 0 = auto), grid target
// (0 = auto), non-temporal flags (bit 0 loads, bit 1 stores), interleaved
// column assignment.
int spx_set_elim_variant(spx_ctx* ctx, int R, int target_wgs, int nt_flags, int interleave) {
  if (!ctx) return SPX_E_ARG;
  // bits 8-10 (flush variant) and 13 (dynamic claims) selected flush kernels
  // that measured slower and were removed: only 0 remains
  CHECK_ARG(((interleave >> 8) & 7) == 0 && ((interleave >> 13) & 1) == 0,
            "flush variant must be 0 (the LDS-DMA ring); block map bits 11-12 only");
  ctx->tune_R = R;
  ctx->tune_wgs = target_wgs;
  ctx->tune_nt = nt_flags < 0 ? -1 : (nt_flags & 3);
  ctx->elim_ilv = interleave & 1;
  ctx->elim_pipe = (interleave & 2) ? 0 : 1;  // bit 1 of `interleave`: disable pipelining
  ctx->elim_xcd = (interleave & 4) ? 1 : 0;   // bit 2: XCD-aware block swizzle
  ctx->flush_map = (interleave >> 11) & 3;    // bits 11-12: flush block map
  choose_geometry(ctx);  // also resolves the automatic nt flags
  if (ctx->loaded) {
    if (ctx->rch > ctx->nbr) {  // ratio_part must hold rch partials
      dfree(ctx->ratio_part);
      HIPC(hipMalloc(&ctx->ratio_part, sizeof(Key) * ratio_part_len(ctx)));
    }
  }
  drop_graphs(ctx);
  return SPX_OK;
}

int spx_get_row(spx_ctx* ctx, int64_t i, double* out) {
  if (!ctx) return SPX_E_ARG;
  if (int rc = rp_recover(ctx)) return rc;
  CHECK_ARG(ctx->loaded && out && i >= 0 && i < ctx->m_local, "bad row");
  HIPC(hipSetDevice(ctx->device));
  double* d = nullptr;
  HIPC(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(double) * ctx->N, ctx->stream));
  hipLaunchKernelGGL(get_row_kernel, dim3(ctx->nbn), dim3(BLK), 0, ctx->stream, ctx->A, ctx->ld,
                     ctx->N, i, d);
  HIPC(hipGetLastError());
  HIPC(hipMemcpyAsync(out, d, sizeof(double) * ctx->N, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipFreeAsync(d, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  return SPX_OK;
}

int spx_set_phase2_objective(spx_ctx* ctx, const double* cost) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(ctx->loaded && cost, "no tableau / null cost");
  CHECK_ARG(!ctx->sharded, "phase-2 objective of a sharded tableau is not supported");
  HIPC(hipSetDevice(ctx->device));
  double* d = nullptr;
  const size_t nc = (size_t)std::max<int64_t>(1, ctx->N - 1);
  HIPC(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(double) * nc, ctx->stream));
  HIPC(hipMemcpyAsync(d, cost, sizeof(double) * (ctx->N - 1), hipMemcpyHostToDevice,
                      ctx->stream));
  hipLaunchKernelGGL(phase2_obj_kernel, dim3(ctx->nbn), dim3(BLK), 0, ctx->stream, ctx->A,
                     ctx->ld, ctx->m_local, ctx->N, d, ctx->basis, ctx->obj);
  HIPC(hipGetLastError());
  HIPC(hipFreeAsync(d, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  return SPX_OK;
}

// Variant actually in use: R, rch, G, nt flags, interleave, pipeline, ld.
int spx_get_elim_variant(const spx_ctx* ctx, int64_t out[7]) {
  if (!ctx || !out) return SPX_E_ARG;
  out[0] = ctx->R;
  out[1] = ctx->rch;
  out[2] = ctx->G;
  out[3] = ctx->elim_nt;
  out[4] = ctx->elim_ilv;
  out[5] = ctx->elim_pipe | (ctx->elim_xcd << 1);
  out[6] = ctx->ld;
  return SPX_OK;
}

// Pivot chain of a window: mode 0 = one persistent launch per window when the
// tableau fits (<= 512 x CUs columns and rows; single-GPU contexts), 1 = two
// launches per pivot (lazy_ratio -> lazy_norm), 2 / 3 = the persistent chain
// with 256- / 512-thread blocks.  min_blocks raises the persistent grid above
// its minimum (tuning; 0 = minimum).  (Round 4's one-XCD chains, modes 4 and
// 5, measured slower than mode 0 on every A/B and were removed in round 5:
// DESIGN.md §4b.)
int spx_set_chain(spx_ctx* ctx, int mode, int min_blocks) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(mode >= 0 && mode <= 3 && min_blocks >= 0 && min_blocks <= CHAIN_MAX_BLOCKS,
            "chain mode must be 0..3 (modes 4 / 5 were removed), min_blocks 0..256");
  ctx->chain_mode = mode;
  ctx->chain_min_blocks = min_blocks;
  drop_graphs(ctx);
  return SPX_OK;
}

// Blocks of the persistent chain for the loaded tableau (0: not used).
int spx_get_chain(spx_ctx* ctx, int* blocks) {
  if (!ctx || !blocks) return SPX_E_ARG;
  *blocks = ctx->loaded && ctx->win_k ? chain_blocks(ctx, nullptr, true) : 0;
  return SPX_OK;
}

// Process-wide budget of persistent-chain blocks in flight on `device`
// (admission); blocks < 0 restores the default (SPX_CHAIN_BUDGET,
// else the device's CU count).
int spx_set_chain_budget(int device, int blocks) {
  ChainAdmission& a = adm();
  std::lock_guard<std::mutex> lk(a.mu);
  if (blocks < 0) a.budget.erase(device);
  else a.budget[device] = blocks;
  return SPX_OK;
}

// Admission record of a context: calls run with the persistent chain, calls
// refused (launch-per-phase chain instead), blocks it holds right now.
int spx_get_chain_stats(spx_ctx* ctx, int64_t out[3]) {
  if (!ctx || !out) return SPX_E_ARG;
  ChainAdmission& a = adm();
  std::lock_guard<std::mutex> lk(a.mu);
  out[0] = ctx->chain_calls[0];
  out[1] = ctx->chain_calls[1];
  out[2] = ctx->adm_blocks;
  return SPX_OK;
}

// Window flush in use: variant (bits 8-10 of spx_set_elim_variant's
// interleave), block map (bits 11-12), and the row chunks / column groups of
// the last flush launch (0 before the first).
int spx_get_flush_variant(const spx_ctx* ctx, int64_t out[4]) {
  if (!ctx || !out) return SPX_E_ARG;
  out[0] = 0;  // the LDS-DMA ring (the only flush since round 3)
  out[1] = ctx->flush_map;
  out[2] = ctx->last_flush_rch;
  out[3] = ctx->last_flush_G;
  return SPX_OK;
}

// Path of the cross-process admission table of `device` (DESIGN.md §4b,
// "Admission"), e.g. for an operator to inspect or clear it.
int spx_chain_shm_path(int device, char* out, int cap) {
  if (!out || cap <= 0) return SPX_E_ARG;
  const std::string p = shm_path(device);
  if ((int)p.size() >= cap) return SPX_E_ARG;
  std::memcpy(out, p.c_str(), p.size() + 1);
  return SPX_OK;
}

// Start handshake of persistent chains (spx_chain.hpp chain_start): bound in
// us (0 = automatic: 20 us on one GPU, 100 ms for row shards); < 0 makes every
// persistent window abort at its start, so the call reruns it (test hook).
int spx_set_chain_handshake(spx_ctx* ctx, int64_t us) {
  if (!ctx) return SPX_E_ARG;
  // (-k: abort every k-th window; k must fit the device's 32-bit modulo)
  CHECK_ARG(us >= -(int64_t)INT32_MAX && us <= (int64_t)1 << 40, "handshake bound out of range");
  ctx->hs_us = us;
  return SPX_OK;
}

// Windows this context reran after their persistent chain found its blocks
// not co-resident (ST_NOTRES).
int spx_get_chain_reruns(spx_ctx* ctx, int64_t* n) {
  if (!ctx || !n) return SPX_E_ARG;
  *n = ctx->chain_reruns;
  return SPX_OK;
}

// Leaving-row transport of the row-sharded chain for the next
// spx_peer_import / spx_peer_chain_local: 0 pull, 1 owner-push.
int spx_set_peer_push(spx_ctx* ctx, int on) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(on == 0 || on == 1, "peer push must be 0 (pull) or 1 (owner-push)");
  ctx->peer_push = on;
  return SPX_OK;
}

// The transport of the imported peer chain (-1: none imported).
int spx_get_peer_push(spx_ctx* ctx, int* on) {
  if (!ctx || !on) return SPX_E_ARG;
  *on = ctx->peer_ok ? ctx->peers.push : -1;
  return SPX_OK;
}

// Diagnostic: this rank's exported buffers and the peer
// pointers it imported.  out[0] tableau, out[1] record buffer, out[2] import
// generation, then per rank q < nranks: out[3 + 2q] tableau, out[4 + 2q]
// record buffer as mapped here (0 when not imported).
int spx_peer_debug(spx_ctx* ctx, uint64_t* out, int n) {
  if (!ctx || !out) return SPX_E_ARG;
  CHECK_ARG(n >= 3 + 2 * ctx->nranks, "spx_peer_debug: out too small");
  out[0] = (uint64_t)(uintptr_t)ctx->A;
  out[1] = (uint64_t)(uintptr_t)ctx->gr_ratio;
  out[2] = ctx->peer_gen;
  for (int q = 0; q < ctx->nranks; ++q) {
    out[3 + 2 * q] = ctx->peer_ok ? (uint64_t)(uintptr_t)ctx->peers.A[q] : 0;
    out[4 + 2 * q] = ctx->peer_ok ? (uint64_t)(uintptr_t)ctx->peers.ratio[q] : 0;
  }
  return SPX_OK;
}

// Diagnostic: out[0] buffers this context ever exported, out[1]
// buffers in its pool, out[2] ever-exported buffers still held (pooled or the
// current load's): out[0] == out[2] while none was freed.  n >= 3.
int spx_peer_pool_debug(spx_ctx* ctx, uint64_t* out, int n) {
  if (!ctx || !out) return SPX_E_ARG;
  CHECK_ARG(n >= 3, "spx_peer_pool_debug: out too small");
  uint64_t held = 0;
  for (void* p : ctx->ever_exported) {
    bool h = p == (void*)ctx->A || p == (void*)ctx->gr_ratio;
    for (const auto& e : ctx->pool) h |= e.p == p;
    held += h ? 1 : 0;
  }
  out[0] = ctx->ever_exported.size();
  out[1] = ctx->pool.size();
  out[2] = held;
  return SPX_OK;
}

int spx_peer_groups(spx_ctx* ctx, int* ngroups, int* group, int* members) {
  if (!ctx || !ngroups || !group || !members) return SPX_E_ARG;
  if (!ctx->peer_ok) {
    ctx->err = "spx_peer_groups: no imported peer chain";
    return SPX_E_STATE;
  }
  *ngroups = ctx->peers.ngroups;
  *group = ctx->peers.group;
  *members = ctx->peer_same_dev;
  return SPX_OK;
}

// Layout knob: extra doubles per column; takes effect at the next load.
int spx_set_ld_pad(spx_ctx* ctx, int pad) {
  if (!ctx) return SPX_E_ARG;
  CHECK_ARG(pad == -1 || (pad >= 0 && pad % 2 == 0 && pad <= 4096),
            "ld pad must be -1 (auto) or even, 0..4096");
  ctx->ld_pad = pad;
  return SPX_OK;
}

}  // extern "C"
