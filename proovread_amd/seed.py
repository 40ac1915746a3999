"""Seeding front end (C-ABI pr_seed_*: host path, and the GPU path pr_seed_gpu_*): `bwa-proovread index` + the seeding and
chaining part of `bwa-proovread mem` (bin/proovread:1270, 1313), which produce the
seed-extension task list of the SW stage.  See include/prgpu.h and DESIGN.md
(parity with bwa-proovread unpinned)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi


class SeedOpts(C.Structure):
    _fields_ = [("min_seed_len", C.c_int), ("min_chain_weight", C.c_int), ("w", C.c_int),
                ("split_factor", C.c_double), ("split_width", C.c_int), ("max_mem_intv", C.c_int),
                ("max_occ", C.c_int), ("drop_ratio", C.c_double), ("max_chain_gap", C.c_int),
                ("mask_level", C.c_double), ("a", C.c_int), ("o_del", C.c_int), ("e_del", C.c_int),
                ("o_ins", C.c_int), ("e_ins", C.c_int), ("b", C.c_int)]


class SeedTask(C.Structure):
    _fields_ = [(k, C.c_int32) for k in ("sr", "lr", "strand", "qbeg", "rbeg", "slen", "rmax0", "rmax1",
                                          "chain", "rank")]


class SeedTasks(C.Structure):
    _fields_ = [("n", C.c_int64), ("t", C.POINTER(SeedTask))]


TASK_DTYPE = np.dtype([(k, np.int32) for k, _ in SeedTask._fields_])
_done = False


def _setup(L):
    global _done
    if _done:
        return
    L.pr_seed_opts_default.argtypes = [C.POINTER(SeedOpts), C.c_int]
    L.pr_seed_opts_default.restype = None
    L.pr_seed_index_build.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
    L.pr_seed_index_free.argtypes = [C.c_void_p]
    L.pr_seed_index_free.restype = None
    L.pr_seed_map.argtypes = [C.c_void_p, C.POINTER(SeedOpts), C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                              C.POINTER(SeedTasks)]
    L.pr_seed_tasks_free.argtypes = [C.POINTER(SeedTasks)]
    L.pr_seed_tasks_free.restype = None
    L.pr_seed_index_digest.argtypes = [C.c_void_p, C.c_void_p]
    L.pr_seed_index_occ.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_int64)]
    L.pr_seed_smem.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_void_p, C.c_void_p,
                               C.c_void_p, C.c_int, C.POINTER(C.c_int)]
    L.pr_seed_map_device_caps.argtypes = [C.c_void_p, C.POINTER(SeedOpts), C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                          C.POINTER(SeedTasks), C.c_void_p]
    L.pr_seed_gpu_upload.argtypes = [C.c_void_p, C.c_void_p]
    L.pr_seed_gpu_map.argtypes = [C.c_void_p, C.POINTER(SeedOpts), C.c_void_p, C.c_void_p, C.c_int,
                                  C.POINTER(SeedTasks), C.c_void_p]
    L.pr_seed_gpu_last_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    L.pr_seed_gpu_index_build.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    L.pr_seed_gpu_index_digest.argtypes = [C.c_void_p, C.c_void_p]
    L.pr_seed_gpu_index_last_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    L.pr_seed_gpu_phase_ticks.argtypes = [C.c_void_p, C.c_void_p]
    L.pr_seed_gpu_pass2_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    L.pr_seed_gpu_pass2_reads.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    L.pr_seed_gpu_seed_count.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    _done = True


def default_opts(finish: bool = False) -> SeedOpts:
    L = _abi.lib()
    _setup(L)
    o = SeedOpts()
    L.pr_seed_opts_default(C.byref(o), 1 if finish else 0)
    return o


class SeedIndex:
    """Index of a long-read shard (nt4 pool + offsets), both strands."""

    def __init__(self, lr_seq: np.ndarray, lr_off: np.ndarray):
        self.L = _abi.lib()
        _setup(self.L)
        self._seq = np.ascontiguousarray(lr_seq, np.uint8)
        self._off = np.ascontiguousarray(lr_off, np.int64)
        h = C.c_void_p()
        _abi.check(self.L.pr_seed_index_build(self._seq.ctypes.data, self._off.ctypes.data, len(self._off) - 1,
                                              C.byref(h)), "pr_seed_index_build")
        self.h = h

    def close(self):
        if self.h:
            self.L.pr_seed_index_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def digest(self) -> tuple:
        """Digests of the index tables (pr_seed_index_digest)."""
        out = np.zeros(6, np.uint64)
        _abi.check(self.L.pr_seed_index_digest(self.h, out.ctypes.data), "pr_seed_index_digest")
        return tuple(int(x) for x in out)

    def occ(self, s: np.ndarray) -> int:
        s = np.ascontiguousarray(s, np.uint8)
        n = C.c_int64()
        _abi.check(self.L.pr_seed_index_occ(self.h, s.ctypes.data, len(s), C.byref(n)), "pr_seed_index_occ")
        return n.value

    def smem(self, q: np.ndarray, x: int, min_intv: int = 1):
        q = np.ascontiguousarray(q, np.uint8)
        cap = len(q) + 1
        st, en, oc = np.zeros(cap, np.int32), np.zeros(cap, np.int32), np.zeros(cap, np.int64)
        n = C.c_int()
        ret = self.L.pr_seed_smem(self.h, q.ctypes.data, len(q), x, min_intv, st.ctypes.data, en.ctypes.data,
                                  oc.ctypes.data, cap, C.byref(n))
        if ret < 0:
            _abi.check(ret, "pr_seed_smem")
        return [(int(st[i]), int(en[i]), int(oc[i])) for i in range(n.value)], ret

    def map(self, sr_seq: np.ndarray, sr_off: np.ndarray, opts: SeedOpts | None = None, threads: int = 0):
        """Seed-extension tasks (structured array, TASK_DTYPE) in read order, chain order."""
        opts = opts or default_opts()
        sr_seq = np.ascontiguousarray(sr_seq, np.uint8)
        sr_off = np.ascontiguousarray(sr_off, np.int64)
        out = SeedTasks()
        _abi.check(self.L.pr_seed_map(self.h, C.byref(opts), sr_seq.ctypes.data, sr_off.ctypes.data,
                                      len(sr_off) - 1, threads, C.byref(out)), "pr_seed_map")
        return self._take(out)

    def map_device_caps(self, sr_seq: np.ndarray, sr_off: np.ndarray, opts: SeedOpts | None = None,
                        threads: int = 0):
        """The GPU path's core and fixed scratch capacities run on the host -> (tasks, status per read)."""
        opts = opts or default_opts()
        sr_seq = np.ascontiguousarray(sr_seq, np.uint8)
        sr_off = np.ascontiguousarray(sr_off, np.int64)
        st = np.zeros(max(1, len(sr_off) - 1), np.int32)
        out = SeedTasks()
        _abi.check(self.L.pr_seed_map_device_caps(self.h, C.byref(opts), sr_seq.ctypes.data, sr_off.ctypes.data,
                                                  len(sr_off) - 1, threads, C.byref(out), st.ctypes.data),
                   "pr_seed_map_device_caps")
        return self._take(out), st[:len(sr_off) - 1]

    def to_gpu(self, ctx: "_abi.Context"):
        """Copy the index into the context's HBM (pr_seed_gpu_upload)."""
        _abi.check(self.L.pr_seed_gpu_upload(ctx.h, self.h), "pr_seed_gpu_upload")
        self._ctx = ctx

    def map_gpu(self, sr_seq: np.ndarray, sr_off: np.ndarray, opts: SeedOpts | None = None,
                allow_flagged: bool = False):
        """Seeding on the GPU -> (tasks, status per read).  Reads flagged with a scratch overflow
        have no tasks; unless allow_flagged, that raises."""
        return _map_gpu(self.L, self._ctx, sr_seq, sr_off, opts, allow_flagged)

    def gpu_ms(self) -> float:
        return _last_ms(self.L.pr_seed_gpu_last_ms, self._ctx)

    def phase_ms(self) -> dict:
        return _phase_ms(self.L, self._ctx)

    def seed_count(self) -> int:
        """Seeds of the last map (kept in HBM with keep_on_device)."""
        n = C.c_int64()
        _abi.check(self.L.pr_seed_gpu_seed_count(self._ctx.h, C.byref(n)), "pr_seed_gpu_seed_count")
        return n.value

    def _take(self, out: SeedTasks):
        return _take(self.L, out)


def _take(L, out: SeedTasks):
    try:
        n = int(out.n)
        if n == 0:
            return np.zeros(0, TASK_DTYPE)
        buf = C.cast(out.t, C.POINTER(C.c_int32 * (10 * n))).contents
        return np.frombuffer(bytes(buf), dtype=TASK_DTYPE).copy()
    finally:
        L.pr_seed_tasks_free(C.byref(out))


def _last_ms(fn, ctx) -> float:
    v = C.c_double()
    _abi.check(fn(ctx.h, C.byref(v)), fn.__name__)
    return v.value


def _count(L, ctx) -> int:
    """Seeds of the context's last pr_seed_gpu_map."""
    n = C.c_int64()
    _abi.check(L.pr_seed_gpu_seed_count(ctx.h, C.byref(n)), "pr_seed_gpu_seed_count")
    return n.value


def _phase_ms(L, ctx) -> dict:
    """Wave time per part of the last GPU seeding launch (ms summed over waves)."""
    t = np.zeros(4, np.uint64)
    _abi.check(L.pr_seed_gpu_phase_ticks(ctx.h, t.ctypes.data), "pr_seed_gpu_phase_ticks")
    n2 = C.c_int64()
    _abi.check(L.pr_seed_gpu_pass2_reads(ctx.h, C.byref(n2)), "pr_seed_gpu_pass2_reads")
    out = {k: round(float(v) / 1e5, 1) for k, v in
           zip(("occ_table", "lane_phase_and_pass2_smems", "pass2_chaining", "pass2_filter_out"), t)}
    out["pass2_reads"] = n2.value
    lt = np.zeros(6, np.uint64)
    L.pr_seed_gpu_lane_ticks.argtypes = [C.c_void_p, C.c_void_p]
    _abi.check(L.pr_seed_gpu_lane_ticks(ctx.h, lt.ctypes.data), "pr_seed_gpu_lane_ticks")
    out["pass1_lane_ms_summed"] = {k: round(float(v) / 1e5, 1) for k, v in
                                   zip(("smem_pass", "reseeding", "y_seeds_sort", "chaining", "chain_flt", "output"), lt)}
    if hasattr(L, "pr_seed_gpu_occ_ticks"):   # (older builds of the library, PRGPU_LIB A/B runs)
        ot = np.zeros(3, np.uint64)
        L.pr_seed_gpu_occ_ticks.argtypes = [C.c_void_p, C.c_void_p]
        _abi.check(L.pr_seed_gpu_occ_ticks(ctx.h, ot.ctypes.data), "pr_seed_gpu_occ_ticks")
        out["occ_table_parts"] = {k: round(float(v) / 1e5, 1) for k, v in zip(("starts", "hits", "count_table"), ot)}
    if hasattr(L, "pr_seed_gpu_pass2_ticks"):
        t2 = np.zeros(7, np.uint64)
        L.pr_seed_gpu_pass2_ticks.argtypes = [C.c_void_p, C.c_void_p]
        _abi.check(L.pr_seed_gpu_pass2_ticks(ctx.h, t2.ctypes.data), "pr_seed_gpu_pass2_ticks")
        out["pass2_parts"] = {"one_lane_reads": int(t2[0])}
        out["pass2_parts"].update({k: round(float(v) / 1e5, 1) for k, v in
                                   zip(("chain_wave", "chain_one_lane", "chain_flt", "max_read_occ_table",
                                        "max_read_smems", "max_read"), t2[1:])})
    p2 = C.c_double()
    _abi.check(L.pr_seed_gpu_pass2_ms(ctx.h, C.byref(p2)), "pr_seed_gpu_pass2_ms")
    out["pass2_wall_ms"] = round(p2.value, 1)
    return out


def _map_gpu(L, ctx, sr_seq, sr_off, opts, allow_flagged, keep_on_device=False):
    opts = opts or default_opts()
    sr_seq = np.ascontiguousarray(sr_seq, np.uint8)
    sr_off = np.ascontiguousarray(sr_off, np.int64)
    st = np.zeros(max(1, len(sr_off) - 1), np.int32)
    if keep_on_device:   # the seeds stay in HBM for iteration.Iteration(gpu_seeds=True)
        rc = L.pr_seed_gpu_map(ctx.h, C.byref(opts), sr_seq.ctypes.data, sr_off.ctypes.data, len(sr_off) - 1,
                               None, st.ctypes.data)
        if rc != 0 and not (allow_flagged and rc == -9):
            _abi.check(rc, "pr_seed_gpu_map")
        return None, st[:len(sr_off) - 1]
    out = SeedTasks()
    rc = L.pr_seed_gpu_map(ctx.h, C.byref(opts), sr_seq.ctypes.data, sr_off.ctypes.data, len(sr_off) - 1,
                           C.byref(out), st.ctypes.data)
    if rc != 0 and not (allow_flagged and rc == -9):
        L.pr_seed_tasks_free(C.byref(out))
        _abi.check(rc, "pr_seed_gpu_map")
    return _take(L, out), st[:len(sr_off) - 1]


class DeviceSeedIndex:
    """The index of a long-read shard built in the context's HBM (pr_seed_gpu_index_build:
    the host build's tables, byte for byte) and seeding against it (pr_seed_gpu_map)."""

    def __init__(self, ctx: "_abi.Context", lr_seq: np.ndarray, lr_off: np.ndarray):
        self.L = _abi.lib()
        _setup(self.L)
        self._ctx = ctx
        seq = np.ascontiguousarray(lr_seq, np.uint8)
        off = np.ascontiguousarray(lr_off, np.int64)
        _abi.check(self.L.pr_seed_gpu_index_build(ctx.h, seq.ctypes.data, off.ctypes.data, len(off) - 1),
                   "pr_seed_gpu_index_build")

    def digest(self) -> tuple:
        out = np.zeros(6, np.uint64)
        _abi.check(self.L.pr_seed_gpu_index_digest(self._ctx.h, out.ctypes.data), "pr_seed_gpu_index_digest")
        return tuple(int(x) for x in out)

    def build_ms(self) -> float:
        return _last_ms(self.L.pr_seed_gpu_index_last_ms, self._ctx)

    def map(self, sr_seq: np.ndarray, sr_off: np.ndarray, opts: SeedOpts | None = None, allow_flagged: bool = False,
            keep_on_device: bool = False):
        """-> (seeds or None when keep_on_device, status per read)."""
        return _map_gpu(self.L, self._ctx, sr_seq, sr_off, opts, allow_flagged, keep_on_device)

    def gpu_ms(self) -> float:
        return _last_ms(self.L.pr_seed_gpu_last_ms, self._ctx)

    def phase_ms(self) -> dict:
        return _phase_ms(self.L, self._ctx)

    def seed_count(self) -> int:
        """Seeds of the last map (kept in HBM with keep_on_device)."""
        n = C.c_int64()
        _abi.check(self.L.pr_seed_gpu_seed_count(self._ctx.h, C.byref(n)), "pr_seed_gpu_seed_count")
        return n.value
