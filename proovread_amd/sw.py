"""Seed-extension stage host layer: the ksw part of `bwa-proovread mem`
(bin/proovread:1313) run by libprgpu.so for a batch of (short read, long read,
seed) tasks.  Output fields follow bwa's mem_alnreg_t / mem_aln_t
(qb, qe, rb, re, score = AS:i, truesc, pos, CIGAR)."""
from __future__ import annotations

import ctypes as C
import dataclasses
from typing import Optional

import numpy as np

from . import _abi

NT4 = np.full(256, 4, np.uint8)
for _i, _c in enumerate(b"ACGT"):
    NT4[_c] = _i
    NT4[ord(chr(_c).lower())] = _i


def to_nt4(s: str) -> np.ndarray:
    return NT4[np.frombuffer(s.encode("latin-1"), np.uint8)]


class SwOpts(C.Structure):
    _fields_ = [("a", C.c_int32), ("b", C.c_int32), ("o_del", C.c_int32), ("e_del", C.c_int32),
                ("o_ins", C.c_int32), ("e_ins", C.c_int32), ("w", C.c_int32), ("pen_clip5", C.c_int32),
                ("pen_clip3", C.c_int32), ("zdrop", C.c_int32), ("min_score_per_base", C.c_double),
                ("bin_size", C.c_int32), ("bin_length", C.c_double), ("drop_ratio", C.c_double),
                ("mask_level", C.c_double), ("mask_level_redun", C.c_double), ("max_chain_gap", C.c_int32)]


class SwBatch(C.Structure):
    _fields_ = [("n_sr", C.c_int32), ("sr_off", _abi.P64), ("sr_seq", _abi.PU8), ("n_lr", C.c_int32),
                ("lr_off", _abi.P64), ("lr_seq", _abi.PU8), ("n_task", C.c_int64), ("t_sr", _abi.P32),
                ("t_lr", _abi.P32), ("t_strand", _abi.PU8), ("t_qbeg", _abi.P32), ("t_rbeg", _abi.P32),
                ("t_slen", _abi.P32), ("t_chain", _abi.P32), ("read_id0", C.c_int64)]


class SwOut(C.Structure):
    _fields_ = [("qb", _abi.P32), ("qe", _abi.P32), ("rb", _abi.P32), ("re", _abi.P32), ("score", _abi.P32),
                ("truesc", _abi.P32), ("pos", _abi.P32), ("ncigar", _abi.P32), ("pass_", _abi.PU8),
                ("status", _abi.P32), ("cigar_off", _abi.P64), ("cigar", _abi.PU32), ("cigar_cap", C.c_int64),
                ("task", _abi.P32), ("flag", _abi.P32)]


def _setup(L):
    if getattr(L, "_sw_ready", False):
        return
    L.pr_sw_opts_default.argtypes = [C.POINTER(SwOpts), C.c_int]
    L.pr_sw_run.argtypes = [C.c_void_p, C.POINTER(SwOpts), C.POINTER(SwBatch), C.POINTER(SwOut)]
    L.pr_sw_upload.argtypes = [C.c_void_p, C.POINTER(SwBatch)]
    L.pr_sw_launch.argtypes = [C.c_void_p, C.POINTER(SwOpts)]
    L.pr_sw_download.argtypes = [C.c_void_p, C.POINTER(SwOut)]
    L.pr_sw_last_timing.argtypes = [C.c_void_p, _abi.PD, _abi.PD]
    L.pr_sw_last_cells.argtypes = [C.c_void_p, _abi.P64, _abi.P64]
    L.pr_sw_dominant_kernel.argtypes = [C.c_void_p, _abi.PD, _abi.P64]
    L.pr_sw_extension_kernels.argtypes = [C.c_void_p, _abi.PD, _abi.P64, _abi.P32]
    L.pr_sw_phase_cycles.argtypes = [C.c_void_p, _abi.P64]
    L.pr_sw_cigar_total.argtypes = [C.c_void_p, _abi.P64, _abi.P64]
    L.pr_sw_aln_count.argtypes = [C.c_void_p, _abi.P64]
    L.pr_sw_bwa_stats.argtypes = [C.c_void_p, _abi.P32, _abi.P64, _abi.P64]
    L._sw_ready = True


def default_opts(finish: bool = False) -> SwOpts:
    L = _abi.lib()
    _setup(L)
    o = SwOpts()
    L.pr_sw_opts_default(C.byref(o), 1 if finish else 0)
    return o


@dataclasses.dataclass
class SwInput:
    sr_off: np.ndarray   # int64 [n_sr+1]
    sr_seq: np.ndarray   # uint8 nt4
    lr_off: np.ndarray   # int64 [n_lr+1]
    lr_seq: np.ndarray   # uint8 nt4
    t_sr: np.ndarray     # int32
    t_lr: np.ndarray     # int32
    t_strand: np.ndarray  # uint8
    t_qbeg: np.ndarray   # int32
    t_rbeg: np.ndarray   # int32
    t_slen: np.ndarray   # int32
    # bwa mode: the tasks are pr_seed_map's seeds (grouped by short read, then chain, in
    # rank order) and t_chain their chain index; outputs are the reported alignments
    t_chain: Optional[np.ndarray] = None
    read_id0: int = 0

    def c_batch(self) -> SwBatch:
        P = _abi.ptr
        b = SwBatch()
        b.n_sr = len(self.sr_off) - 1
        b.sr_off = P(self.sr_off, C.c_int64)
        b.sr_seq = P(self.sr_seq, C.c_uint8)
        b.n_lr = len(self.lr_off) - 1
        b.lr_off = P(self.lr_off, C.c_int64)
        b.lr_seq = P(self.lr_seq, C.c_uint8)
        b.n_task = len(self.t_sr)
        b.t_sr = P(self.t_sr, C.c_int32)
        b.t_lr = P(self.t_lr, C.c_int32)
        b.t_strand = P(self.t_strand, C.c_uint8)
        b.t_qbeg = P(self.t_qbeg, C.c_int32)
        b.t_rbeg = P(self.t_rbeg, C.c_int32)
        b.t_slen = P(self.t_slen, C.c_int32)
        if self.t_chain is not None:
            b.t_chain = P(self.t_chain, C.c_int32)
            b.read_id0 = int(self.read_id0)
        return b


class SwResult:
    """Per-task outputs (bwa mode: per reported alignment, SAM order, with the seed `task`
    that made it and the SAM `flag` bits); CIGARs variable length, compacted in order
    (cigar_off prefix)."""

    def __init__(self, n: int):
        self.a = {k: np.zeros(max(n, 1), np.int32) for k in
                  ("qb", "qe", "rb", "re", "score", "truesc", "pos", "ncigar", "status", "task", "flag")}
        self.a["pass"] = np.zeros(max(n, 1), np.uint8)
        self.a["cigar_off"] = np.zeros(n + 1, np.int64)
        self.a["cigar"] = np.zeros(1, np.uint32)
        o = SwOut()
        P = _abi.ptr
        for k in ("qb", "qe", "rb", "re", "score", "truesc", "pos", "ncigar", "status", "task", "flag"):
            setattr(o, k, P(self.a[k], C.c_int32))
        o.pass_ = P(self.a["pass"], C.c_uint8)
        o.cigar_off = P(self.a["cigar_off"], C.c_int64)
        self.c = o
        self.n = n
        self.n_overflow = 0

    def size_cigar(self, total: int):
        self.a["cigar"] = np.zeros(max(total, 1), np.uint32)
        self.c.cigar = _abi.ptr(self.a["cigar"], C.c_uint32)
        self.c.cigar_cap = total

    def __getitem__(self, k):
        return self.a[k][: self.n] if k not in ("cigar", "cigar_off") else self.a[k]

    def cigar_ops(self, t: int) -> np.ndarray:
        o = self.a["cigar_off"]
        return self.a["cigar"][int(o[t]):int(o[t + 1])]

    def cigar_str(self, t: int) -> str:
        return "".join(f"{int(x) >> 4}{'MIDNSHP=X'[int(x) & 15]}" for x in self.cigar_ops(t))


def run(inp: SwInput, opts: Optional[SwOpts] = None, ctx: Optional[_abi.Context] = None) -> SwResult:
    L = _abi.lib()
    _setup(L)
    ctx = ctx or _abi.default_context()
    opts = opts or default_opts()
    b = inp.c_batch()
    _abi.check(L.pr_sw_upload(ctx.h, C.byref(b)), "pr_sw_upload")
    _abi.check(L.pr_sw_launch(ctx.h, C.byref(opts)), "pr_sw_launch")
    na = C.c_int64()
    _abi.check(L.pr_sw_aln_count(ctx.h, C.byref(na)), "pr_sw_aln_count")
    res = SwResult(na.value)
    tot, nov = C.c_int64(), C.c_int64()
    _abi.check(L.pr_sw_cigar_total(ctx.h, C.byref(tot), C.byref(nov)), "pr_sw_cigar_total")
    res.size_cigar(tot.value)
    res.n_overflow = nov.value
    _abi.check(L.pr_sw_download(ctx.h, C.byref(res.c)), "pr_sw_download")
    return res


def bwa_stats(ctx: _abi.Context):
    """bwa mode: (extension rounds, seeds extended, mem_patch_reg scores) of the last launch."""
    L = _abi.lib()
    _setup(L)
    r, n, p = C.c_int32(), C.c_int64(), C.c_int64()
    _abi.check(L.pr_sw_bwa_stats(ctx.h, C.byref(r), C.byref(n), C.byref(p)), "pr_sw_bwa_stats")
    return r.value, n.value, p.value


def bwa_timing(ctx: _abi.Context):
    """bwa mode: (walk ms summed over rounds, main-stream final passes ms, early final pass ms)
    of the last launch (pr_sw_bwa_timing)."""
    L = _abi.lib()
    L.pr_sw_bwa_timing.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
    w, f, e = C.c_float(), C.c_float(), C.c_float()
    _abi.check(L.pr_sw_bwa_timing(ctx.h, C.byref(w), C.byref(f), C.byref(e)), "pr_sw_bwa_timing")
    return w.value, f.value, e.value


def last_timing(ctx: _abi.Context):
    L = _abi.lib()
    _setup(L)
    a, b = C.c_double(), C.c_double()
    L.pr_sw_last_timing(ctx.h, C.byref(a), C.byref(b))
    ce, cg = C.c_int64(), C.c_int64()
    L.pr_sw_last_cells(ctx.h, C.byref(ce), C.byref(cg))
    return a.value, b.value, ce.value, cg.value


def dominant_kernel(ctx: _abi.Context):
    """(ms, cells) of the last launch's dominant kernel: the CIGAR pass's packed launch."""
    L = _abi.lib()
    _setup(L)
    ms, cells = C.c_double(), C.c_int64()
    _abi.check(L.pr_sw_dominant_kernel(ctx.h, C.byref(ms), C.byref(cells)), "pr_sw_dominant_kernel")
    return ms.value, cells.value


def extension_kernels(ctx: _abi.Context):
    """(summed ms, DP cells, launches) of every extension DP launch of the last launch."""
    L = _abi.lib()
    _setup(L)
    ms, cells, n = C.c_double(), C.c_int64(), C.c_int32()
    _abi.check(L.pr_sw_extension_kernels(ctx.h, C.byref(ms), C.byref(cells), C.byref(n)), "pr_sw_extension_kernels")
    return ms.value, cells.value, n.value


def phase_cycles(ctx: _abi.Context):
    """Wave-cycle totals of the packed CIGAR kernel's phases (masks, DP, backtrack, emit)."""
    L = _abi.lib()
    _setup(L)
    out = (C.c_int64 * 4)()
    _abi.check(L.pr_sw_phase_cycles(ctx.h, out), "pr_sw_phase_cycles")
    return list(out)
