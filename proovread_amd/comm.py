"""Collectives of the multi-rank correction loop (one process per GPU).

The reference has no distributed backend: bin/proovread fans work out to processes on
one host and joins them through files.  Across the GPUs of a node the
loop exchanges:

  * the per-iteration masked-fraction statistic {bpt, bpN} (all-reduce; input of
    mask_shortcut_frac, bin/proovread:1702-1720, 2026-2047) — on the device;
  * in the exact-parity layout, seed-extension tasks (all-to-all to the long-read
    owners) and the corrected / masked reads (all-gather for the next index).

Two interchangeable implementations:

  RcclComm   the product's: RCCL linked into libprgpu (pr_comm_*), on the same HIP
             runtime as the kernels — torch is never loaded into a GPU process.
             Rank 0's RCCL id reaches the other ranks through a file rendezvous
             (single node: all ranks share /tmp), keyed by the launcher's pid and
             MASTER_PORT so concurrent jobs cannot meet.
  TorchComm  torch.distributed (gloo) for the CPU multi-process tests.
"""
from __future__ import annotations

import ctypes as C
import os
import time
from pathlib import Path
from typing import List, Optional, Sequence

import numpy as np

ID_BYTES = 128
DT_I64, DT_F64, DT_I32, DT_U8 = 0, 1, 2, 3
RED_SUM, RED_MAX, RED_MIN = 0, 1, 2


# ---------------------------------------------------------------------------- rendezvous
def rendezvous_path(key: Optional[str] = None) -> Path:
    """The file through which rank 0 publishes the RCCL id.  All ranks of a job are
    children of one launcher (torch.distributed.run's agent, or a test's spawner), so
    the parent pid + MASTER_PORT + run id name the job, and the elastic restart count names
    the attempt (a file an earlier attempt left behind is never read by a later one)."""
    if key is None:
        key = os.environ.get("PRGPU_RDZV_KEY") or "_".join(
            [str(os.getppid()), os.environ.get("MASTER_PORT", "0"), os.environ.get("TORCHELASTIC_RUN_ID", "none"),
             os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")])
    base = Path(os.environ.get("PRGPU_RDZV_DIR", "/tmp"))
    return base / f"prgpu_rdzv_{key}.id"


def publish(path: Path, payload: bytes) -> None:
    tmp = path.with_suffix(f".tmp{os.getpid()}")
    tmp.write_bytes(payload)
    os.replace(tmp, path)   # atomic: readers never see a partial id


def wait_for(path: Path, size: int, timeout: float = 300.0) -> bytes:
    t0 = time.monotonic()
    while True:
        try:
            b = path.read_bytes()
            if len(b) == size:
                return b
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"rendezvous: {path} did not appear within {timeout:.0f} s")
        time.sleep(0.02)


def exchange_id(rank: int, make_id, key: Optional[str] = None, timeout: float = 300.0) -> bytes:
    """Rank 0 creates the id (make_id()) and publishes it; the others read it."""
    path = rendezvous_path(key)
    if rank == 0:
        idb = make_id()
        publish(path, idb)
        return idb
    return wait_for(path, ID_BYTES, timeout)


def _unpack_lists(parts: Sequence[bytes]) -> List[bytes]:
    out: List[bytes] = []
    for p in parts:
        k = int(np.frombuffer(p[:8], np.int64)[0])
        ln = np.frombuffer(p[8:8 + 8 * k], np.int64)
        o = 8 + 8 * k
        for x in ln:
            out.append(p[o:o + int(x)])
            o += int(x)
    return out


def _pack_list(items: Sequence[bytes]) -> bytes:
    lens = np.array([len(x) for x in items], np.int64).tobytes()
    return np.int64(len(items)).tobytes() + lens + b"".join(items)


class _Base:
    rank: int
    world: int

    def allgather_lists(self, items: List[bytes]) -> List[bytes]:
        """Concatenation over ranks (rank order) of per-rank lists of byte strings."""
        return _unpack_lists(self.allgather_bytes(_pack_list(items)))

    def allgather_bytes(self, blob: bytes) -> List[bytes]:   # pragma: no cover - interface
        raise NotImplementedError

    def alltoallv_rows(self, send: np.ndarray, send_counts: np.ndarray) -> np.ndarray:
        """All-to-all of the rows of a 2-D int32 array: send_counts[r] rows (consecutive,
        in rank order) go to rank r; returns the received rows, source-rank-major."""
        send = np.ascontiguousarray(send, dtype=np.int32)
        ncol = send.shape[1]
        got = self.alltoallv_bytes(send.tobytes(), np.asarray(send_counts, np.int64) * 4 * ncol)
        return np.frombuffer(got, np.int32).reshape(-1, ncol).copy()


# ---------------------------------------------------------------------------- RCCL (product)
class RcclComm(_Base):
    """pr_comm_* of libprgpu on a context (one rank per GPU)."""

    def __init__(self, ctx, rank: int, world: int, key: Optional[str] = None):
        from . import _abi
        self.L = _abi.lib()
        L = self.L
        _setup(L)
        self.ctx, self.rank, self.world = ctx, rank, world

        def make_id() -> bytes:
            b = C.create_string_buffer(ID_BYTES)
            _abi.check(L.pr_comm_unique_id(b), "pr_comm_unique_id")
            return b.raw

        idb = exchange_id(rank, make_id, key)
        h = C.c_void_p()
        _abi.check(L.pr_comm_init(ctx.h, world, rank, idb, C.byref(h)), "pr_comm_init")
        self.h = h
        if rank == 0:   # every rank has read the id once the communicator exists on all of them
            self.barrier()
            try:
                rendezvous_path(key).unlink()
            except FileNotFoundError:
                pass
        else:
            self.barrier()

    @classmethod
    def from_env(cls, ctx) -> "RcclComm":
        return cls(ctx, int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")))

    def _chk(self, rc, what):
        from . import _abi
        _abi.check(rc, what)

    def close(self):
        if getattr(self, "h", None):
            self.L.pr_comm_destroy(self.h)
            self.h = None

    def barrier(self):
        self._chk(self.L.pr_comm_barrier(self.h), "pr_comm_barrier")

    def allreduce_dev(self, dev_ptr: int, n: int, dtype: int = DT_I64, op: int = RED_SUM):
        """In-place all-reduce of a device buffer, asynchronous on the context stream."""
        self._chk(self.L.pr_comm_allreduce_dev(self.h, dev_ptr, dev_ptr, n, dtype, op), "pr_comm_allreduce_dev")

    def allreduce_ints(self, vals: Sequence[int], op: int = RED_SUM) -> List[int]:
        a = np.array(list(vals), np.int64)
        self._chk(self.L.pr_comm_allreduce_host(self.h, a.ctypes.data, len(a), DT_I64, op), "pr_comm_allreduce_host")
        return [int(x) for x in a]

    def allreduce_floats(self, vals: Sequence[float], op: int = RED_SUM) -> List[float]:
        a = np.array(list(vals), np.float64)
        self._chk(self.L.pr_comm_allreduce_host(self.h, a.ctypes.data, len(a), DT_F64, op), "pr_comm_allreduce_host")
        return [float(x) for x in a]

    def allgather_bytes(self, blob: bytes) -> List[bytes]:
        counts = (C.c_int64 * self.world)()
        self._chk(self.L.pr_comm_allgatherv_host(self.h, blob, len(blob), None, 0, counts), "pr_comm_allgatherv_host")
        tot = sum(counts)
        out = C.create_string_buffer(max(tot, 1))
        self._chk(self.L.pr_comm_allgatherv_host(self.h, blob, len(blob), out, tot, counts), "pr_comm_allgatherv_host")
        raw = out.raw[:tot]
        parts, o = [], 0
        for c in counts:
            parts.append(raw[o:o + c])
            o += c
        return parts

    def alltoallv_bytes(self, send: bytes, send_counts: np.ndarray) -> bytes:
        sc = np.ascontiguousarray(send_counts, np.int64)
        rc = np.zeros(self.world, np.int64)
        P = C.POINTER(C.c_int64)
        self._chk(self.L.pr_comm_alltoall_counts(self.h, sc.ctypes.data_as(P), rc.ctypes.data_as(P)),
                  "pr_comm_alltoall_counts")
        out = C.create_string_buffer(max(int(rc.sum()), 1))
        self._chk(self.L.pr_comm_alltoallv_host(self.h, send, sc.ctypes.data_as(P), out, rc.ctypes.data_as(P)),
                  "pr_comm_alltoallv_host")
        return out.raw[:int(rc.sum())]


def _setup(L):
    if getattr(L, "_comm_ready", False):
        return
    L.pr_comm_unique_id.argtypes = [C.c_char_p]
    L.pr_comm_init.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_char_p, C.POINTER(C.c_void_p)]
    L.pr_comm_destroy.argtypes = [C.c_void_p]
    L.pr_comm_allreduce_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int]
    L.pr_comm_allreduce_host.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int]
    L.pr_comm_barrier.argtypes = [C.c_void_p]
    L.pr_comm_allgatherv_host.argtypes = [C.c_void_p, C.c_char_p, C.c_int64, C.c_void_p, C.c_int64,
                                          C.POINTER(C.c_int64)]
    L.pr_comm_alltoall_counts.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.pr_comm_alltoallv_host.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_int64), C.c_void_p,
                                         C.POINTER(C.c_int64)]
    L.pr_comm_group_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.pr_comm_group_destroy.argtypes = [C.c_void_p]
    L.pr_comm_group_abort.argtypes = [C.c_void_p]
    L.pr_comm_group_abort.restype = None
    L.pr_comm_init_local.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
    L._comm_ready = True


class LocalGroup:
    """pr_comm_group: `world` ranks as threads of this process, one context each (include/prgpu.h
    pr_comm_init_local) -- the multi-rank device paths on a single GPU."""

    def __init__(self, world: int):
        from . import _abi
        self.L = _abi.lib()
        _setup(self.L)
        self.world = world
        h = C.c_void_p()
        _abi.check(self.L.pr_comm_group_create(world, C.byref(h)), "pr_comm_group_create")
        self.h = h

    def abort(self):
        """A rank left its collective sequence: the ranks waiting in (or later entering) a
        collective return an error instead of waiting forever (pr_comm_group_abort)."""
        if getattr(self, "h", None):
            self.L.pr_comm_group_abort(self.h)

    def close(self):
        if getattr(self, "h", None):
            self.L.pr_comm_group_destroy(self.h)
            self.h = None


class LocalComm(RcclComm):
    """A rank of a LocalGroup: the RcclComm interface over the in-process group's collectives."""

    def __init__(self, ctx, group: LocalGroup, rank: int):
        from . import _abi
        self.L = _abi.lib()
        _setup(self.L)
        self.ctx, self.rank, self.world = ctx, rank, group.world
        h = C.c_void_p()
        _abi.check(self.L.pr_comm_init_local(ctx.h, group.h, rank, C.byref(h)), "pr_comm_init_local")
        self.h = h


# ---------------------------------------------------------------------------- torch (CPU tests)
class TorchComm(_Base):
    """torch.distributed (gloo) implementation, for world_size > 1 tests on CPU."""

    def __init__(self, group=None, device: Optional[str] = None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device

    def _dev(self):
        import torch
        return torch.device(self.device) if self.device else torch.device("cpu")

    def barrier(self):
        self.dist.barrier(group=self.group)

    def allreduce_ints(self, vals: Sequence[int], op: int = RED_SUM) -> List[int]:
        import torch
        t = torch.tensor(list(vals), dtype=torch.int64, device=self._dev())
        ops = {RED_SUM: self.dist.ReduceOp.SUM, RED_MAX: self.dist.ReduceOp.MAX, RED_MIN: self.dist.ReduceOp.MIN}
        self.dist.all_reduce(t, op=ops[op], group=self.group)
        return [int(x) for x in t.cpu().tolist()]

    def allgather_bytes(self, blob: bytes) -> List[bytes]:
        import torch
        n = self.world
        size = torch.tensor([len(blob)], dtype=torch.int64, device=self._dev())
        sizes = [torch.zeros_like(size) for _ in range(n)]
        self.dist.all_gather(sizes, size, group=self.group)
        sz = [int(x.item()) for x in sizes]
        cap = max(max(sz), 1)
        buf = torch.zeros(cap, dtype=torch.uint8)
        if blob:
            buf[:len(blob)] = torch.from_numpy(np.frombuffer(blob, np.uint8).copy())
        buf = buf.to(self._dev())
        outs = [torch.empty(cap, dtype=torch.uint8, device=self._dev()) for _ in range(n)]
        self.dist.all_gather(outs, buf, group=self.group)
        return [outs[r][:sz[r]].cpu().numpy().tobytes() for r in range(n)]

    def alltoallv_bytes(self, send: bytes, send_counts: np.ndarray) -> bytes:
        import torch
        dev = self._dev()
        sc = torch.from_numpy(np.ascontiguousarray(send_counts, np.int64)).to(dev)
        rc = torch.empty_like(sc)
        self.dist.all_to_all_single(rc, sc, group=self.group)
        recv_counts = [int(x) for x in rc.cpu().tolist()]
        src = torch.from_numpy(np.frombuffer(send, np.uint8).copy()).to(dev)
        out = torch.empty(sum(recv_counts), dtype=torch.uint8, device=dev)
        self.dist.all_to_all_single(out, src, recv_counts, [int(x) for x in send_counts], group=self.group)
        return out.cpu().numpy().tobytes()
