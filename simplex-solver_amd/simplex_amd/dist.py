"""Row-sharded tableau across GPUs: one process per GPU.

Partitioning: constraint rows 0..m-1 are split into contiguous blocks, one per
rank, tiling 0..m in rank order; the objective row and the basis are
replicated.  Every rank chooses the entering column locally (identical
objective rows give identical choices, no collective).  The leaving row is the
one real exchange of a pivot, and two protocols implement it, bit-identical to
one GPU and to each other:

* the row-sharded persistent chain (the default at N > 1, ``enable_peer_chain``):
  one launch per window on every rank; each block's ratio record is written to
  every rank's record buffer over xGMI (system-scope granules) and polled
  locally, and the leaving row's stale values are read from its owner's
  tableau through a peer pointer (IPC-mapped across processes).  No RCCL call
  per pivot.
* the RCCL fallback (``set_chain(1)``): per pivot ONE all-gather of every
  rank's [best (ratio, tie, row) key | that row normalised]; every rank takes
  the lexicographic winner (the leaving-row "allreduce-min" RCCL has no MINLOC
  for) and its row (the owner's broadcast without a host-known root).

torch.distributed only ships small host objects: the 128-byte RCCL unique id
and the peer chain's IPC blobs (any backend: gloo on CPU).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L
from .engine import DeviceTableau


def row_partition(m: int, world: int, rank: int) -> tuple:
    """Contiguous near-equal block [row0, row1) of rank `rank`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(m, world)
    row0 = rank * base + min(rank, extra)
    return row0, row0 + base + (1 if rank < extra else 0)


def choose_row_transport(ms_pull: float, ms_push: float | None, push_ok: bool = True) -> str:
    """The leaving-row transport of the row-sharded chain, from a short timed
    trial of each (bench.py): "push" when its self-test passed and its windows
    ran faster, else "pull".  Every rank passes the same (all-reduced) times,
    so every rank makes the same choice."""
    if push_ok and ms_push is not None and ms_push < ms_pull:
        return "push"
    return "pull"


def make_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    rc = L.lib().spx_comm_unique_id(buf)
    if rc != 0:
        raise RuntimeError(f"spx_comm_unique_id failed ({rc})")
    return buf.raw


def exchange_unique_id(make_id=make_unique_id, group=None) -> bytes:
    """Rank 0 creates the id, every rank returns it (torch.distributed)."""
    import torch.distributed as dist
    obj = [make_id() if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    uid = obj[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != 128:
        raise RuntimeError("bad RCCL unique id received")
    return bytes(uid)


class ShardedTableau(DeviceTableau):
    """This rank's row block of a tableau sharded over `world` GPUs."""

    def __init__(self, device: int, rank: int, world: int, uid: bytes | None = None,
                 local: bool | str = False):
        """local=True: the ranks are threads of this process sharing GPUs
        (in-process loopback exchange instead of RCCL; for tests).
        local="peer": no communicator at all; the ranks exchange only through
        the row-sharded persistent chain (enable_peer_chain is then required)."""
        super().__init__(device, _sharded=(rank, world, uid, local))
        self.rank, self.world, self.local = rank, world, local

    def enable_peer_chain(self, allgather=None, push: bool | None = None) -> bool:
        """Set up the row-sharded persistent chain for the loaded rows (DESIGN.md
        §5): every rank calls this after its load.  Virtual ranks meet in
        process; otherwise this rank's blob (IPC handles of its tableau and
        record buffer) is all-gathered with `allgather(bytes) -> list[bytes]`
        (default: torch.distributed.all_gather_object) and imported.
        push: the leaving-row transport (None: keep the context's setting;
        False pull from the owner's tableau, True owner-push into every peer's
        inbox; every rank must pass the same).  Calling it again re-imports,
        e.g. to switch the transport between windows.  Returns True, or False
        when a rank's pool of exported buffers is full for this load
        (SPX_E_NOPEER, the same on every rank): the windows then run the RCCL
        path -- a peer-only shard (local="peer") has none and raises."""
        lib = self._lib
        if push is not None:
            self.set_peer_push(push)
        if self.local is True:
            self._check(lib.spx_peer_chain_local(self._ctx), "spx_peer_chain_local")
            return True
        size = lib.spx_peer_blob_size()
        buf = ctypes.create_string_buffer(size)
        self._check(lib.spx_peer_export(self._ctx, buf, size), "spx_peer_export")
        if allgather is None:
            import torch.distributed as tdist

            def allgather(blob):
                out = [None] * tdist.get_world_size()
                tdist.all_gather_object(out, blob)
                return out
        blobs = allgather(buf.raw)
        if len(blobs) != self.world or any(len(b) != size for b in blobs):
            raise RuntimeError("peer chain: bad blob exchange")
        rc = lib.spx_peer_import(self._ctx, b"".join(blobs), self.world)
        if rc == L.SPX_E_NOPEER and self.local is False:
            return False
        self._check(rc, "spx_peer_import")
        return True

    def set_peer_push(self, on: bool) -> None:
        """Leaving-row transport for the next enable_peer_chain (spx_set_peer_push)."""
        self._check(self._lib.spx_set_peer_push(self._ctx, 1 if on else 0), "spx_set_peer_push")

    def peer_push(self) -> int:
        """The imported peer chain's transport: 0 pull, 1 push, -1 none."""
        v = ctypes.c_int()
        self._check(self._lib.spx_get_peer_push(self._ctx, ctypes.byref(v)), "spx_get_peer_push")
        return int(v.value)

    def peer_debug(self) -> dict:
        """Diagnostic: this rank's exported buffers, the import generation and
        the peer pointers it mapped (spx_peer_debug)."""
        n = 3 + 2 * self.world
        out = (ctypes.c_uint64 * n)()
        self._check(self._lib.spx_peer_debug(self._ctx, out, n), "spx_peer_debug")
        return {"A": out[0], "records": out[1], "gen": out[2],
                "peer_A": [out[3 + 2 * q] for q in range(self.world)],
                "peer_records": [out[4 + 2 * q] for q in range(self.world)]}

    def peer_pool_debug(self) -> dict:
        """Diagnostic: buffers this context ever exported, buffers in its pool,
        and the ever-exported ones it still holds (spx_peer_pool_debug; an
        exported buffer is never freed before close, so held == exported)."""
        out = (ctypes.c_uint64 * 3)()
        self._check(self._lib.spx_peer_pool_debug(self._ctx, out, 3), "spx_peer_pool_debug")
        return {"exported": out[0], "pooled": out[1], "held": out[2]}

    def peer_groups(self) -> dict:
        """Diagnostic: the imported peer chain's device groups (spx_peer_groups)."""
        g, me, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._check(self._lib.spx_peer_groups(self._ctx, ctypes.byref(g), ctypes.byref(me),
                                              ctypes.byref(n)), "spx_peer_groups")
        return {"groups": g.value, "group": me.value, "members": n.value}

    @classmethod
    def from_env(cls, device: int | None = None, group=None) -> "ShardedTableau":
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = exchange_unique_id(group=group)
        return cls(rank if device is None else device, rank, world, uid)

    def load_shard(self, T_rows: np.ndarray, obj: np.ndarray, basis: np.ndarray, m_global: int,
                   row0: int) -> "ShardedTableau":
        return self.load_rows(T_rows, obj, basis, m_global, row0)
