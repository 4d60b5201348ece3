/*
 * spx.h — C-ABI of the MI355X dense simplex pivot engine (libspx.so).
 *
 * This is the drop-in boundary for the tableau-pivoting hot path of
 * the-utn-team/simplex-solver.  In the reference that path is the third-party
 * `simple_simplex==0.0.3` engine, driven from
 *   app/controllers/solver_controller.py:290-319  (_run_simple_simplex:
 *       create_tableau / add_constraint / add_objective / optimize_json_format)
 * and its pivot history is consumed at solver_controller.py:322-363.
 * The Python module `simplex_amd.simple_simplex` re-exposes those four names on
 * top of the entry points below (binding: simplex_amd/_lib.py).
 *
 * Conventions
 *  - Plain pointers and sizes only; no torch types.
 *  - The caller owns every host buffer; the library copies in/out and never
 *    keeps a host pointer after a call returns.  A context owns all device
 *    memory (and the RCCL communicator of a sharded context); spx_destroy
 *    frees it.
 *  - Re-entrant: no global mutable state besides two mutex-guarded registries
 *    (virtual-rank groups, persistent-chain admission per device).  One
 *    context per solve, one HIP stream per context; distinct contexts may be
 *    used from distinct threads concurrently (the reference's /solve is
 *    entered from many threads, tests/test_performance_load.py:80-83).
 *  - Tableau (the spec): rows 0..m-1 are constraints, the
 *    objective row is logically row m ("z_j - c_j" form of a MAX problem, RHS
 *    = current objective value).  Columns 0..N-2 are variables, column N-1 is
 *    the right-hand side.  basis[i] = index of the variable basic in row i.
 *  - Return codes: >= 0 is a solve status with the same numbering as scipy's
 *    OptimizeResult.status (which solver_controller.py:404 maps):
 *       SPX_OPTIMAL 0, SPX_ITER_LIMIT 1, SPX_INFEASIBLE 2, SPX_UNBOUNDED 3;
 *    plain calls return SPX_OK (0).  Negative values are errors; the message
 *    is available from spx_last_error(ctx).
 */
#ifndef SPX_H_
#define SPX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPX_ABI_VERSION 1

/* status / return codes */
#define SPX_OK 0
#define SPX_OPTIMAL 0
#define SPX_ITER_LIMIT 1
#define SPX_INFEASIBLE 2
#define SPX_UNBOUNDED 3
#define SPX_RUNNING 4 /* spx_pivot: a pivot was made, not finished */
#define SPX_E_ARG (-1)
#define SPX_E_HIP (-2)
#define SPX_E_RCCL (-3)
#define SPX_E_STATE (-4)
#define SPX_E_OOM (-5)
#define SPX_E_NOPEER (-6) /* spx_peer_import: this load cannot run the peer chain (a rank's
                           * exported-buffer pool is full); the RCCL path runs instead */

/* pivot rules */
#define SPX_RULE_DANTZIG 0 /* most negative reduced cost, lowest column on ties; lowest row on ratio ties */
#define SPX_RULE_BLAND 1   /* lowest column with rc < -eps_opt; lowest basic-variable index on ratio ties */

/* layouts of host tableau buffers */
#define SPX_ROW_MAJOR 0 /* element (i,j) at buf[i*ld + j] */
#define SPX_COL_MAJOR 1 /* element (i,j) at buf[j*ld + i] */

typedef struct spx_ctx spx_ctx;

typedef struct spx_opts {
  int32_t rule;          /* SPX_RULE_* */
  int32_t skip_zero_cols;/* 1 (default): columns with p[j]==0 are left untouched (bit-identical
                            to the dense update up to the sign of zero); 0: dense sweep */
  double eps_opt;        /* optimality tolerance on reduced costs (default 1e-9) */
  double eps_piv;        /* minimum pivot-column entry for the ratio test (default 1e-12) */
  int64_t max_iters;     /* pivots allowed in this call (<=0: unlimited) */
  double time_limit_s;   /* wall-clock limit (<=0: none); checked between pivot chunks */
  int64_t n_enter;       /* columns [0, n_enter) may enter; <=0 means all but the RHS */
  int32_t chunk;         /* pivots per hipGraph replay (<=0: default 32) */
  int32_t use_graph;     /* 1 (default): replay captured pivot chunks; 0: direct launches */
} spx_opts;

typedef struct spx_result {
  int32_t status;        /* SPX_OPTIMAL / SPX_ITER_LIMIT / SPX_UNBOUNDED */
  int32_t pad;
  int64_t iters;         /* pivots made by this call */
  double objective;      /* tableau objective-row RHS (value of the MAX form) */
  double elapsed_s;      /* wall time of the call */
} spx_result;

/* Fill *o with the defaults documented above. */
void spx_default_opts(spx_opts* o);

/* ---- context lifetime ---------------------------------------------------- */
int spx_create(spx_ctx** out, int device);
int spx_destroy(spx_ctx* ctx);
const char* spx_last_error(const spx_ctx* ctx);
int spx_abi_version(void);

/* ---- sharded (multi-GPU) contexts: one process per GPU, RCCL over xGMI ---- */
/* Writes the 128-byte RCCL unique id (rank 0 creates it; the caller ships it
 * to the other ranks, e.g. with torch.distributed over gloo/TCP). */
int spx_comm_unique_id(char out_id[128]);
/* Like spx_create, but joins a communicator of nranks contexts; rank r will
 * own a contiguous block of constraint rows (given at load time). */
int spx_create_sharded(spx_ctx** out, int device, int rank, int nranks, const char id[128]);
/* Same as spx_create_sharded, but the ranks are contexts of ONE process (one
 * host thread per rank, any devices, up to 16 ranks) joined by the 128-byte
 * group id, exchanging through device copies instead of RCCL.  Used to test
 * the sharded path on a single GPU; not capturable in a hipGraph. */
int spx_create_sharded_local(spx_ctx** out, int device, int rank, int nranks,
                             const char id[128]);

/* Like spx_create_sharded, but with no communicator: the ranks (processes or
 * threads, on one or several GPUs, at most 16) exchange only through the
 * row-sharded persistent chain set up by spx_peer_export / spx_peer_import, so
 * such a context must run windowed (spx_set_window) with the persistent chain. */
int spx_create_sharded_peer(spx_ctx** out, int device, int rank, int nranks);

/* ---- row-sharded persistent chain -------------------------- */
/* After every rank loaded its rows, the ranks' windows can run ONE persistent
 * launch per window (the single-GPU chain, spx_chain.hpp) instead of three
 * launches and an RCCL all-gather per pivot: each block's ratio record is
 * written to every rank's record buffer and polled locally, and the leaving
 * row's stale values are read from its owner's tableau through a peer
 * pointer.  Across processes the peers are IPC-mapped: spx_peer_export writes
 * this rank's blob (spx_peer_blob_size() bytes), the caller all-gathers the
 * blobs (e.g. torch.distributed over gloo) and every rank calls
 * spx_peer_import with all of them in rank order.  Virtual ranks of one
 * process call spx_peer_chain_local instead.  Valid until the next load; the
 * chain is used when its grid fits (every rank's blocks in one poll, the
 * chains sharing a GPU all resident), else the RCCL path runs. */
int spx_peer_blob_size(void);
int spx_peer_export(spx_ctx* ctx, void* out, int64_t cap);
/* Collective: every rank imports after every rank exported.  The buffers a
 * context exported are never freed before spx_destroy: a
 * reload moves them to the context's pool, and later loads of that context
 * reuse the smallest pooled buffer that fits (at most 4 per buffer role; a
 * load that would need a fifth gets plain buffers that are never exported:
 * spx_peer_import then returns SPX_E_NOPEER on every rank, the windows of
 * that load run the RCCL path where a communicator exists, and the next load
 * frees them -- round 5 failed the load instead).  spx_destroy of an exported context waits (bounded, 10 s) for
 * every peer to release its IPC mapping, so the ranks should destroy
 * together. */
int spx_peer_import(spx_ctx* ctx, const void* blobs, int nranks);
int spx_peer_chain_local(spx_ctx* ctx);
/* Leaving-row transport of the row-sharded chain, for the next
 * spx_peer_import / spx_peer_chain_local (every rank must choose the same, or
 * the import fails): 0 = pull (default; every rank reads the owner's row
 * through a peer pointer, scattered 8-byte system-scope loads over xGMI),
 * 1 = owner-push (the owner's blocks write its row contiguously into
 * every peer's inbox; north_star's "single broadcast of the pivot row").
 * Bit-identical either way.  spx_get_peer_push: the imported chain's
 * transport (-1: no peer chain imported). */
int spx_set_peer_push(spx_ctx* ctx, int on);
int spx_get_peer_push(spx_ctx* ctx, int* on);
/* Diagnostic: out[0] this rank's tableau, out[1] its record buffer, out[2]
 * the import generation, then for every rank q the tableau and record buffer
 * pointers as mapped here (out[3+2q], out[4+2q]; 0 before an import).
 * n >= 3 + 2 * nranks. */
int spx_peer_debug(spx_ctx* ctx, uint64_t* out, int n);
/* Diagnostic: out[0] buffers this context ever exported, out[1] buffers in its
 * pool, out[2] ever-exported buffers it still holds (pooled or loaded); an
 * exported buffer is never freed before spx_destroy, so out[0] == out[2].
 * n >= 3. */
int spx_peer_pool_debug(spx_ctx* ctx, uint64_t* out, int n);
/* Diagnostic (round 6): the device groups of the imported peer chain (ranks
 * sharing a GPU; each group settles its own start handshake, then waits for
 * the other groups' verdicts), this rank's group and its member count.
 * SPX_PEER_GROUP_TAG (a test hook, read at spx_peer_export) splits ranks of
 * one GPU into groups.  SPX_E_STATE before an import. */
int spx_peer_groups(spx_ctx* ctx, int* ngroups, int* group, int* members);

/* ---- data in / out ------------------------------------------------------- */
/* Load a full tableau of `rows` = m+1 rows (objective row LAST) and `cols` = N
 * columns; basis has m entries.  ld is the host leading dimension. */
int spx_load(spx_ctx* ctx, const double* T, int64_t rows, int64_t cols, int64_t ld,
             int layout, const int64_t* basis);
/* Sharded load: this rank's constraint rows [row0, row0+m_local) of a tableau
 * with m_global constraint rows, the (replicated) objective row `obj` (N
 * values) and the full basis (m_global entries).  Also valid for 1 rank. */
int spx_load_rows(spx_ctx* ctx, const double* A, int64_t m_local, int64_t cols, int64_t ld,
                  int layout, const double* obj, const int64_t* basis, int64_t m_global,
                  int64_t row0);
/* Replace the objective row (N values), e.g. between phase 1 and phase 2. */
int spx_set_objective(spx_ctx* ctx, const double* obj);
/* Copy out this context's rows (m_local+1 rows, objective row last). */
int spx_get_tableau(spx_ctx* ctx, double* out, int64_t ld, int layout);
int spx_get_objective(spx_ctx* ctx, double* out);      /* N values */
int spx_get_basis(spx_ctx* ctx, int64_t* out);         /* m_global values */
int spx_get_column(spx_ctx* ctx, int64_t j, double* out); /* local rows of column j */
int spx_get_row(spx_ctx* ctx, int64_t i, double* out);    /* N values of local row i */
/* Phase-2 objective row computed on the device from the current tableau:
 * obj = -cost + sum_i cost[basis[i]] * T[i,:] (cost has N-1 entries, RHS
 * cost 0), accumulated in row order (bit-identical to the host formula).
 * Single-GPU contexts only. */
int spx_set_phase2_objective(spx_ctx* ctx, const double* cost);
/* Pivot history of the context since load: up to `cap` (row, col) pairs,
 * returns the number of pivots recorded in *n. */
int spx_get_history(spx_ctx* ctx, int64_t* rc_pairs, int64_t cap, int64_t* n);
int spx_dims(const spx_ctx* ctx, int64_t* m_global, int64_t* m_local, int64_t* cols,
             int64_t* row0);

/* ---- pivoting ------------------------------------------------------------ */
/* Run the pivot loop until optimal / unbounded / limits. */
int spx_solve(spx_ctx* ctx, const spx_opts* opts, spx_result* res);
/* One pivot chosen by the rule.  Returns SPX_RUNNING with *r,*c set when a
 * pivot was made, or SPX_OPTIMAL / SPX_UNBOUNDED (no pivot made). */
int spx_pivot(spx_ctx* ctx, const spx_opts* opts, int64_t* r, int64_t* c);
/* One pivot on a given element (r, c) (used to drive artificial variables out
 * of the basis after phase 1).  T[r,c] must be nonzero. */
int spx_pivot_at(spx_ctx* ctx, int64_t r, int64_t c);
/* Enqueue exactly `npivots` rule-chosen pivots without host synchronisation
 * (benchmark primitive; pivots after termination are no-ops on the device).
 * If `time_elim` = k > 0, HIP events bracket every k-th elimination launch, or
 * in window mode every k-th window's flush; the timed launches are direct, the
 * other windows replay the per-window hipGraph when use_graph is set.  A
 * window whose persistent chain aborted at its start handshake (see
 * spx_set_chain_handshake) is rerun by the next drain of the context
 * (spx_sync, spx_state, a getter, or the next call), so the request still
 * ends after exactly `npivots` pivots.  Two duties follow from not waiting:
 * (1) peer-only row shards (spx_create_sharded_peer) must reach that drain
 * together -- the rerun is again a cross-rank persistent chain.  A rank that
 * drains late is waited for: the early ranks' rerun windows abort at the
 * handshake (100 ms each) and are rerun until it arrives, which the late
 * rank catches up with at once (tested with 0.6 s and 2.5 s lags on one
 * GPU).  The early ranks give up with SPX_E_STATE only after rerunning for 30
 * s (SPX_PEER_RERUN_S; round 5: after 16 aborts, ~1.7 s); ranks on different
 * GPUs (device groups) no longer fault after a ~4 s wait for the other
 * GPUs' verdicts: a group still undecided after the handshake bound is
 * decided ABORT by a compare-and-swap on its verdict word (round 6), so every
 * group aborts that window and reruns it.  bench.py and dist.py drain every rank right after the
 * call, behind a barrier.  (2) The call's persistent-chain admission
 * (spx_set_chain_budget) is held until that drain, or until another call or
 * admission decision of this process sees the call's work complete; a
 * process sharing its GPU with other processes should spx_sync after
 * spx_run_pivots, else their chains may be refused (and run the slower,
 * bit-identical launch-per-phase chain) meanwhile. */
int spx_run_pivots(spx_ctx* ctx, const spx_opts* opts, int64_t npivots, int time_elim);
/* Wait for the context's enqueued work (and finish an spx_run_pivots request
 * whose window had to be rerun). */
int spx_sync(spx_ctx* ctx);
/* Device-side state after spx_sync: status code (SPX_RUNNING while going),
 * total pivots since load, and the objective-row RHS. */
int spx_state(spx_ctx* ctx, int32_t* status, int64_t* iters, double* objective);
/* Sum and count of the elimination-kernel (or flush) event timings collected
 * by spx_run_pivots(..., time_elim=k) since the last reset; `touched_cols`
 * receives the sum, over every pivot (window mode: every flush) since the
 * reset, of the columns the kernel updated (algorithmic-byte accounting). */
int spx_elim_timing(spx_ctx* ctx, double* total_ms, int64_t* count, int64_t* touched_cols,
                    int reset);

/* Tuning knob of the elimination kernel: rows per thread R (2, 4, 8; 0 = auto),
 * grid target (0 = auto), non-temporal flags (bit 0 loads, bit 1 stores; -1 = auto) and
 * `interleave`: bit 0 = interleaved column assignment (else contiguous column
 * ranges), bit 1 = disable software pipelining of column pairs, bit 2 = XCD-aware
 * block swizzle, bits 8-10 = window flush variant (must be 0: the LDS-DMA ring
 * of 12; the register-ring and ring-9/10 variants were removed in round 3),
 * bits 11-12 = window flush block map (bit 11 chunk-major, bit 12 group rotated
 * by row chunk; 0 = group-major, the default; bit 13, the removed dynamically
 * claimed flush, must be 0).  Returns SPX_E_ARG for a removed variant. */
int spx_set_elim_variant(spx_ctx* ctx, int R, int target_wgs, int nt_flags, int interleave);
/* The elimination variant in use: R, row chunks, column groups, nt flags,
 * interleave, pipelining, leading dimension. */
int spx_get_elim_variant(const spx_ctx* ctx, int64_t out[7]);
/* The window flush in use: variant and block map (bits 8-10 / 11-13 of
 * spx_set_elim_variant's `interleave`), then the row chunks and column groups
 * of the last flush launch (0 before the first flush). */
int spx_get_flush_variant(const spx_ctx* ctx, int64_t out[4]);
/* Windowed ("delayed") elimination: apply K pivots per streaming pass over
 * the tableau (K in 2, 4, 8, 12, 16, 24, 28, 32; 0 or 1 = one pass per pivot).
 * Results are bit-identical.  Row-sharded contexts run the
 * same windows with one all-gather per pivot. */
int spx_set_window(spx_ctx* ctx, int K);
/* The row_fix fold: on = 1, a window's fast-path
 * leaving rows are rewritten by the NEXT window's persistent chain launch
 * (each thread its own column, before the start handshake) and after a
 * call's last window by one row_fix launch; on = 0 (default), a row_fix
 * launch after every window.  Single-GPU persistent chains with 256-thread
 * blocks only; bit-identical either way.  Measured no faster on config 3
 * (the fix's ~13 us moves onto the chain's critical path), hence off. */
int spx_set_row_fix_fold(spx_ctx* ctx, int on);
/* Pivot-choice timing (diagnostic): when on, every window records HIP events
 * around its chain (the persistent kernel, or the lazy kernels of its slots);
 * spx_chain_timing returns their sum and count since the last reset.  The
 * event nodes add stream time, so measure it outside a timed region. */
int spx_set_chain_timing(spx_ctx* ctx, int on);
int spx_chain_timing(spx_ctx* ctx, double* total_ms, int64_t* count, int reset);
/* Pivot chain of a window (the K pivot choices before its flush): mode 0
 * (default) runs them as ONE persistent launch when the tableau fits (at most
 * 512 x CUs columns and rows, single-GPU contexts), mode 1 as two
 * launches per pivot, modes 2 / 3 force the persistent chain's 256- / 512-thread
 * blocks; any other mode is SPX_E_ARG (round 4's one-XCD modes 4 / 5 were
 * removed).  Results are bit-identical.  min_blocks (0..256) raises the
 * persistent grid above its minimum (tuning; 0 = minimum). */
int spx_set_chain(spx_ctx* ctx, int mode, int min_blocks);
/* Blocks of the persistent chain the loaded tableau uses (0: not used). */
int spx_get_chain(spx_ctx* ctx, int* blocks);
/* Admission of persistent chains: a persistent chain needs all
 * of its blocks resident at once, so the processes on a device admit chains
 * whose blocks in flight fit a budget (default: the device's CU count, or the
 * SPX_CHAIN_BUDGET environment variable); a call that does not fit runs its
 * windows with the launch-per-phase chain, bit-identical.  This makes the
 * reference's concurrent /solve calls (tests/test_performance_load.py:80,190,268)
 * slow down instead of failing.  blocks < 0 restores the default; 0 forces the
 * launch-per-phase chain. */
int spx_set_chain_budget(int device, int blocks);
/* The budget is shared by every process using the same GPU through a table in
 * /dev/shm (entries {pid, blocks, start time} under flock; entries of dead
 * processes, or of a pid since reused, are free;
 * SPX_CHAIN_SHM=0 turns it off).  This writes the table's path for `device`
 * (at most cap bytes with the terminating NUL). */
int spx_chain_shm_path(int device, char* out, int cap);
/* A context's admission record: out[0] calls run with the persistent chain,
 * out[1] calls refused (launch-per-phase chain), out[2] blocks held now. */
int spx_get_chain_stats(spx_ctx* ctx, int64_t out[3]);
/* Start handshake of persistent chains ("Residency"): before
 * its first store every block of a chain announces itself and waits at most
 * `us` microseconds for all the others (0 = automatic: 20 us on one GPU, 100 ms
 * for row shards, whose ranks enqueue independently).  If some block is not
 * resident (its CU held by another kernel or process, or another chain ahead
 * of it on the same hardware queue), no block stores anything, the window
 * reports ST_NOTRES, and spx_solve / spx_pivot / spx_pivot_at rerun it with
 * the launch-per-phase chain (peer-only shards: the persistent chain again,
 * giving up after 16 CONSECUTIVE aborts of the same pivot), bit-identical.
 * us = -k < 0 makes every k-th window (by window epoch) abort; -1 every
 * window (test hooks). */
int spx_set_chain_handshake(spx_ctx* ctx, int64_t us);
/* Windows the context reran after such an abort. */
int spx_get_chain_reruns(spx_ctx* ctx, int64_t* n);
/* Layout knob: extra doubles of padding per stored column (even, 0..4096);
  * applies to the next spx_load / spx_load_rows; -1 = automatic. */
int spx_set_ld_pad(spx_ctx* ctx, int pad);

#ifdef __cplusplus
}
#endif
#endif /* SPX_H_ */
