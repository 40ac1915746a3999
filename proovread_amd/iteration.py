"""One proovread correction iteration on the GPU (pr_iter_* of libprgpu.so):
seed extension + CIGAR for every (short read, long read) task, the device-side
hand-off into samtools coordinate order, and the consensus of every long read
— bin/proovread:835-869 for one task (run_bwa 1254-1322, create_sorted_bam
1330-1355, correct_sr_mt 1528-1721) without the SAM/BAM files in between."""
from __future__ import annotations

import ctypes as C
from types import SimpleNamespace
from typing import List, Optional

import numpy as np

from . import _abi, cns, sw


class IterBatch(C.Structure):
    _fields_ = [("sw", sw.SwBatch), ("task_lr_off", _abi.P64), ("lr_qual", _abi.PU8), ("ref_seq", _abi.PU8)]


class OwnBatch(C.Structure):
    _fields_ = [("lr0", C.c_int32), ("n_lr", C.c_int32), ("lr_off", _abi.P64), ("ref_seq", _abi.PU8),
                ("lr_qual", _abi.PU8), ("n_sr", C.c_int32), ("sr_off", _abi.P64), ("sr_seq", _abi.PU8),
                ("from_set", C.c_int32)]


def _setup(L):
    if getattr(L, "_iter_ready", False):
        return
    sw._setup(L)
    L.pr_iter_upload.argtypes = [C.c_void_p, C.POINTER(IterBatch)]
    L.pr_iter_upload_gpu_seeds.argtypes = [C.c_void_p, C.POINTER(IterBatch)]
    L.pr_iter_launch.argtypes = [C.c_void_p, C.POINTER(sw.SwOpts), C.POINTER(_abi.CnsParams)]
    L.pr_iter_download.argtypes = [C.c_void_p, C.POINTER(_abi.CnsOut)]
    L.pr_iter_bounds.argtypes = [C.c_void_p, _abi.P32, _abi.P64, C.POINTER(_abi.CnsBounds)]
    L.pr_iter_last_timing.argtypes = [C.c_void_p, _abi.PD, _abi.PD, _abi.PD, _abi.PD]
    L.pr_iter_stats.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
    L.pr_ctx_sync.argtypes = [C.c_void_p]
    L.pr_iter_alignment_stats.argtypes = [C.c_void_p, _abi.P64, _abi.P64, _abi.P64]
    L.pr_sw_upload_gpu_seeds.argtypes = [C.c_void_p, C.POINTER(sw.SwBatch)]
    L.pr_aln_exchange.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, _abi.P64, _abi.P64]
    L.pr_aln_exchange_local.argtypes = [C.c_void_p, C.c_int, _abi.P64, _abi.P64, _abi.P64]
    L.pr_iter_upload_owned.argtypes = [C.c_void_p, C.POINTER(OwnBatch)]
    L.pr_lrset_load.argtypes = [C.c_void_p, C.c_int32, _abi.P64, _abi.PU8, _abi.PU8]
    L.pr_lrset_info.argtypes = [C.c_void_p, _abi.P32, _abi.P64]
    L.pr_lrset_index.argtypes = [C.c_void_p, C.c_int]
    L.pr_lrset_commit.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    L.pr_lrset_download.argtypes = [C.c_void_p, _abi.P64, _abi.PU8, _abi.PU8, _abi.PU8]
    L.pr_iter_upload_lrset.argtypes = [C.c_void_p, C.POINTER(sw.SwBatch)]
    from . import seed
    L.pr_srset_load.argtypes = [C.c_void_p, C.c_int64, _abi.P64, _abi.PU8]
    L.pr_seed_gpu_map_sampled.argtypes = [C.c_void_p, C.POINTER(seed.SeedOpts), _abi.P64, C.c_int, _abi.P32]
    L.pr_srset_sample.argtypes = [C.c_void_p, _abi.P64, C.c_int]
    L.pr_lrset_snapshot.argtypes = [C.c_void_p]
    L.pr_lrset_restore.argtypes = [C.c_void_p]
    L._iter_ready = True


class Iteration:
    """A resident iteration batch on one GPU (upload once, launch many)."""

    def __init__(self, d, lr_qual: Optional[np.ndarray] = None, ctx: Optional[_abi.Context] = None,
                 ref_seq: Optional[np.ndarray] = None, gpu_seeds: bool = False):
        """d: reads + tasks (synth.Dataset fields); lr_qual: the reference qualities (phred+33,
        default '$'); ref_seq: ASCII consensus reference when it differs from the mapped long
        reads d.lr_seq (iterations after the first map to the masked consensus); gpu_seeds: the
        tasks are the seeds the last DeviceSeedIndex.map(keep_on_device=True) left in HBM (d's
        task fields are not used)."""
        self.L = _abi.lib()
        _setup(self.L)
        self.ctx = ctx or _abi.default_context()
        self.d = d
        n_lr = len(d.lr_off) - 1
        self.task_lr_off = np.zeros(n_lr + 1, np.int64)
        if gpu_seeds:
            z = np.zeros(0, np.int32)
            self.inp = sw.SwInput(d.sr_off, d.sr_seq, d.lr_off, d.lr_seq, z, z, np.zeros(0, np.uint8), z, z, z)
        else:
            self.inp = d.sw_input()
            np.cumsum(np.bincount(d.t_lr, minlength=n_lr), out=self.task_lr_off[1:])
        if lr_qual is None:
            lr_qual = np.full(int(d.lr_off[-1]), ord("$"), np.uint8)   # raw CLR reads: phred 3
        self.lr_qual = lr_qual
        if ref_seq is not None:
            ref_seq = np.ascontiguousarray(ref_seq, np.uint8)
            if len(ref_seq) != int(d.lr_off[-1]):
                raise ValueError("ref_seq must have the long reads' layout (lr_off)")
        self.ref_seq = ref_seq
        b = IterBatch()
        b.sw = self.inp.c_batch()
        b.task_lr_off = _abi.ptr(self.task_lr_off, C.c_int64)
        b.lr_qual = _abi.ptr(self.lr_qual, C.c_uint8)
        if ref_seq is not None:
            b.ref_seq = _abi.ptr(self.ref_seq, C.c_uint8)
        self._b = b
        if gpu_seeds:
            _abi.check(self.L.pr_iter_upload_gpu_seeds(self.ctx.h, C.byref(b)), "pr_iter_upload_gpu_seeds")
        else:
            _abi.check(self.L.pr_iter_upload(self.ctx.h, C.byref(b)), "pr_iter_upload")
        nl, nt, bd = C.c_int32(), C.c_int64(), _abi.CnsBounds()
        _abi.check(self.L.pr_iter_bounds(self.ctx.h, C.byref(nl), C.byref(nt), C.byref(bd)), "pr_iter_bounds")
        self.n_lr, self.n_task, self.bounds = nl.value, nt.value, bd
        self.out = None

    def launch(self, sw_opts: sw.SwOpts, params: cns.CnsParams):
        self._pc = params.to_c()
        self._so = sw_opts
        _abi.check(self.L.pr_iter_launch(self.ctx.h, C.byref(sw_opts), C.byref(self._pc)), "pr_iter_launch")

    def sync(self):
        _abi.check(self.L.pr_ctx_sync(self.ctx.h), "pr_ctx_sync")

    def stats_to(self, dev_ptr: int, min_phred: int = 20):
        """Enqueue {corrected bases, bases >= min_phred} into device memory dev_ptr (int64[2])."""
        _abi.check(self.L.pr_iter_stats(self.ctx.h, min_phred, C.c_void_p(dev_ptr)), "pr_iter_stats")

    def mask_to(self, dev_ptr: int, p):
        """Enqueue the masking of the resident consensus (SeqFilter --phred-mask, proovread:1706);
        {bases, N bases} (bpt, bpN) go to device memory dev_ptr (int64[2])."""
        from . import mask
        mask._setup(self.L)
        self._mp = p
        _abi.check(self.L.pr_iter_mask(self.ctx.h, C.byref(p), C.c_void_p(dev_ptr)), "pr_iter_mask")

    def masked(self) -> List[bytes]:
        """Masked consensus of the last mask_to, one bytes object per long read (status 0 reads)."""
        a = self.download()
        buf = np.zeros(self.bounds.seq_cap + 1, np.uint8)
        _abi.check(self.L.pr_iter_mask_download(self.ctx.h, buf.ctypes.data), "pr_iter_mask_download")
        out = []
        for i in range(self.n_lr):
            o, sl = int(a["out_off"][i]), int(a["seq_len"][i])
            out.append(buf[o:o + sl].tobytes() if a["status"][i] == 0 else b"")
        return out

    def _out_buffers(self, bin_size=20.0):
        n = self.n_lr
        lens = np.diff(self.d.lr_off)
        nb = np.floor(lens / bin_size).astype(np.int64) + 1
        a = dict(out_off=np.zeros(n + 1, np.int64), status=np.zeros(n, np.int32), seq_len=np.zeros(n, np.int32),
                 trace_len=np.zeros(n, np.int32), ncigar=np.zeros(n, np.int32), nchim=np.zeros(n, np.int32),
                 seq=np.zeros(self.bounds.seq_cap + 1, np.uint8), qual=np.zeros(self.bounds.seq_cap + 1, np.uint8),
                 trace=np.zeros(self.bounds.seq_cap + 1, np.uint8),
                 cigar=np.zeros(self.bounds.seq_cap + 1, np.uint32), chim_off=np.zeros(n + 1, np.int64),
                 chim=np.zeros(4 * (self.bounds.chim_cap + 1), np.int32),
                 kept=np.zeros(self.n_task + 1, np.uint8), bin_bases=np.zeros(int(nb.sum()) + 1, np.int64))
        o = _abi.CnsOut()
        P = _abi.ptr
        for k, ct in (("out_off", C.c_int64), ("status", C.c_int32), ("seq_len", C.c_int32),
                      ("trace_len", C.c_int32), ("ncigar", C.c_int32), ("nchim", C.c_int32), ("seq", C.c_uint8),
                      ("qual", C.c_uint8), ("trace", C.c_uint8), ("cigar", C.c_uint32), ("chim_off", C.c_int64),
                      ("chim", C.c_int32), ("kept", C.c_uint8), ("bin_bases", C.c_int64)):
            setattr(o, k, P(a[k], ct))
        return a, o

    def download(self, with_arrays: bool = True):
        if self.out is None:
            self.out = self._out_buffers()
        a, o = self.out
        _abi.check(self.L.pr_iter_download(self.ctx.h, C.byref(o)), "pr_iter_download")
        return a

    def alignment_stats(self):
        v = [C.c_int64() for _ in range(3)]
        _abi.check(self.L.pr_iter_alignment_stats(self.ctx.h, *[C.byref(x) for x in v]), "alignment_stats")
        return [x.value for x in v]

    def timing(self):
        v = [C.c_double() for _ in range(4)]
        self.L.pr_iter_last_timing(self.ctx.h, *[C.byref(x) for x in v])
        return [x.value for x in v]

    def cns_phase_ms(self):
        """Consensus workgroup time per phase (ms summed over workgroups) of the last launch."""
        t = (C.c_uint64 * 24)()
        _abi.check(self.L.pr_cns_phase_ticks(self.ctx.h, t, 24), "pr_cns_phase_ticks")
        names = ["prep", "binning", "state_table", "scatter", "argmax_write", "cigar", "chimera", "idle",
                 "scatter_zero", "chimera_tables", "chimera_entropy", "scatter_walk"]
        out = {k: t[i] / 1e5 for i, k in enumerate(names)}
        out.update(groups=int(t[12]), items=int(t[13]), windows=int(t[14]), scatter_prepass=t[15] / 1e5,
                   scatter_ins=t[16] / 1e5, visits=int(t[17]), runs=int(t[18]), ins_states=int(t[19]),
                   scatter_runscan=t[20] / 1e5)
        return out

    def chimeras(self):
        """-> (status, nchim, chim_off, chim rows [from, to, npos, ntot]) per long read: the part
        of the output the finish task keeps on the host (detect_chimera)."""
        n = self.n_lr
        a = dict(status=np.zeros(n, np.int32), nchim=np.zeros(n, np.int32), chim_off=np.zeros(n + 1, np.int64),
                 chim=np.zeros(4 * (self.bounds.chim_cap + 1), np.int32))
        o = _abi.CnsOut()
        for k, ct in (("status", C.c_int32), ("nchim", C.c_int32), ("chim_off", C.c_int64), ("chim", C.c_int32)):
            setattr(o, k, _abi.ptr(a[k], ct))
        _abi.check(self.L.pr_iter_download(self.ctx.h, C.byref(o)), "pr_iter_download")
        return a["status"], a["nchim"], a["chim_off"], a["chim"].reshape(-1, 4)

    def chim_lines(self, ids: List[str]) -> List[str]:
        """bam2cns:488's chimera lines of every long read (ids: theirs, in batch order)."""
        st, nch, c0, rows = self.chimeras()
        if not nch.any():
            return []
        # formatted natively (pr_fmt_chim_lines: the finish task's ~125 k lines at configs[1]
        # took ~40 ms as Python f-strings)
        enc = [x.encode() for x in ids]
        off = np.zeros(len(enc) + 1, np.int64)
        np.cumsum([len(x) for x in enc], out=off[1:])
        pool = np.frombuffer(b"".join(enc) or b"\0", np.uint8)
        L = self.L
        L.pr_fmt_chim_lines.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.POINTER(C.c_void_p), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.pr_buffer_free.argtypes = [C.c_void_p]
        n = min(len(ids), len(nch))
        nch32 = np.ascontiguousarray(nch[:n], np.int32)
        c064 = np.ascontiguousarray(c0[:n + 1], np.int64)
        rows32 = np.ascontiguousarray(rows, np.int32)
        txt, ln, nl = C.c_void_p(), C.c_int64(), C.c_int64()
        _abi.check(L.pr_fmt_chim_lines(n, pool.ctypes.data, off.ctypes.data, nch32.ctypes.data, c064.ctypes.data,
                                       rows32.ctypes.data, C.byref(txt), C.byref(ln), C.byref(nl)), "pr_fmt_chim_lines")
        try:
            s = C.string_at(txt.value, ln.value).decode()
        finally:
            L.pr_buffer_free(txt)
        lines = s.split("\n")
        lines.pop()   # (the text ends with a newline)
        return lines

    def results_range(self, first: int, n: int) -> List[cns.ReadResult]:
        """results() of reads [first, first + n) only (pr_iter_download_range)."""
        L = self.L
        L.pr_iter_download_range.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(_abi.CnsOut)]
        oo = np.zeros(n + 1, np.int64)
        co = np.zeros(n + 1, np.int64)
        _abi.check(L.pr_iter_download_range(self.ctx.h, first, n, C.byref(_abi.CnsOut(out_off=_abi.ptr(oo, C.c_int64),
                                                                                      chim_off=_abi.ptr(co, C.c_int64)))),
                   "pr_iter_download_range")
        cap = int(oo[-1]) + 1
        a = dict(out_off=oo, status=np.zeros(n + 1, np.int32), seq_len=np.zeros(n + 1, np.int32),
                 trace_len=np.zeros(n + 1, np.int32), ncigar=np.zeros(n + 1, np.int32), nchim=np.zeros(n + 1, np.int32),
                 seq=np.zeros(cap, np.uint8), qual=np.zeros(cap, np.uint8), trace=np.zeros(cap, np.uint8),
                 cigar=np.zeros(cap, np.uint32), chim_off=co, chim=np.zeros(4 * (int(co[-1]) + 1), np.int32))
        o = _abi.CnsOut()
        for k, ct in (("out_off", C.c_int64), ("status", C.c_int32), ("seq_len", C.c_int32),
                      ("trace_len", C.c_int32), ("ncigar", C.c_int32), ("nchim", C.c_int32), ("seq", C.c_uint8),
                      ("qual", C.c_uint8), ("trace", C.c_uint8), ("cigar", C.c_uint32), ("chim_off", C.c_int64),
                      ("chim", C.c_int32)):
            setattr(o, k, _abi.ptr(a[k], ct))
        _abi.check(L.pr_iter_download_range(self.ctx.h, first, n, C.byref(o)), "pr_iter_download_range")
        out = []
        for k in range(n):
            st = int(a["status"][k])
            r = cns.ReadResult(f"lr{first + k}", st)
            if st == 0:
                o0 = int(oo[k])
                sl, tl, nc = int(a["seq_len"][k]), int(a["trace_len"][k]), int(a["ncigar"][k])
                r.seq = a["seq"][o0:o0 + sl].tobytes().decode("latin-1")
                r.qual = a["qual"][o0:o0 + sl].tobytes().decode("latin-1")
                r.trace = a["trace"][o0:o0 + tl].tobytes().decode("latin-1")
                r.cigar = [(int(x >> 4), "MID"[int(x & 15)]) for x in a["cigar"][o0:o0 + nc]]
                c0, nch = int(co[k]), int(a["nchim"][k])
                r.chim = [tuple(int(v) for v in row) for row in a["chim"][4 * c0:4 * (c0 + nch)].reshape(-1, 4)]
            out.append(r)
        return out

    def results_of(self, reads) -> List[cns.ReadResult]:
        """results() of the listed reads only."""
        return [self.results_range(int(i), 1)[0] for i in reads]

    def statuses(self) -> np.ndarray:
        """Every read's consensus status of the last launch (pr_iter_download_range)."""
        L = self.L
        L.pr_iter_download_range.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(_abi.CnsOut)]
        st = np.zeros(max(self.n_lr, 1), np.int32)
        _abi.check(L.pr_iter_download_range(self.ctx.h, 0, self.n_lr, C.byref(_abi.CnsOut(status=_abi.ptr(st, C.c_int32)))),
                   "pr_iter_download_range")
        return st[:self.n_lr]

    def results(self) -> List[cns.ReadResult]:
        a = self.download()
        out = []
        for i in range(self.n_lr):
            st = int(a["status"][i])
            r = cns.ReadResult(f"lr{i}", st)
            if st == 0:
                o = int(a["out_off"][i])
                sl, tl, nc = int(a["seq_len"][i]), int(a["trace_len"][i]), int(a["ncigar"][i])
                r.seq = a["seq"][o:o + sl].tobytes().decode("latin-1")
                r.qual = a["qual"][o:o + sl].tobytes().decode("latin-1")
                r.trace = a["trace"][o:o + tl].tobytes().decode("latin-1")
                r.cigar = [(int(x >> 4), "MID"[int(x & 15)]) for x in a["cigar"][o:o + nc]]
                c0, nch = int(a["chim_off"][i]), int(a["nchim"][i])
                r.chim = [tuple(int(v) for v in row) for row in a["chim"][4 * c0:4 * (c0 + nch)].reshape(-1, 4)]
            out.append(r)
        return out


class ShardSW:
    """Exact-parity layout, step 1 on a rank: the bwa-mode SW batch of the short-read shard
    [s, e) whose seeds the last DeviceSeedIndex.map(keep_on_device=True) left in HBM (the index of
    ALL long reads, lr_map / lr_off as mapped), uploaded once; launch() runs the SW on it (sr 0
    of the shard is global id s: bwa's hash ties)."""

    def __init__(self, ctx, sr: np.ndarray, sr_off: np.ndarray, s: int, e: int, lr_map: np.ndarray,
                 lr_off: np.ndarray, device_pools: bool = False):
        """device_pools: the read pools are the device copies the seeding made (the index's long
        reads, the seeded shard) -- no second host upload."""
        self.L = _abi.lib()
        _setup(self.L)
        self.ctx = ctx
        sr_off = np.asarray(sr_off, np.int64)
        self._sh_off = np.ascontiguousarray(sr_off[s:e + 1] - sr_off[s], np.int64)
        self._sh_seq = None if device_pools else np.ascontiguousarray(sr[sr_off[s]:sr_off[e]], np.uint8)
        self._lr_off = np.ascontiguousarray(lr_off, np.int64)
        self._lr_map = None if device_pools else np.ascontiguousarray(lr_map, np.uint8)
        z = np.zeros(0, np.int32)
        inp = sw.SwInput(self._sh_off, self._sh_seq, self._lr_off, self._lr_map, z, z, np.zeros(0, np.uint8), z, z, z)
        b = inp.c_batch()
        b.read_id0 = int(s)
        _abi.check(self.L.pr_sw_upload_gpu_seeds(ctx.h, C.byref(b)), "pr_sw_upload_gpu_seeds")

    def launch(self, sw_opts: sw.SwOpts):
        self._so = sw_opts
        _abi.check(self.L.pr_sw_launch(self.ctx.h, C.byref(sw_opts)), "pr_sw_launch")


def shard_sw(ctx, sw_opts: sw.SwOpts, sr: np.ndarray, sr_off: np.ndarray, s: int, e: int, lr_map: np.ndarray,
             lr_off: np.ndarray) -> None:
    """ShardSW upload + one launch."""
    ShardSW(ctx, sr, sr_off, s, e, lr_map, lr_off).launch(sw_opts)


def exchange(ctx, comm, s: int, bounds: np.ndarray) -> int:
    """Step 2: every reported alignment of the last shard_sw to the owner of its long read
    (pr_aln_exchange: device pack, RCCL all-to-all of device buffers; comm None = world 1).
    Returns the alignments this rank received."""
    L = _abi.lib()
    _setup(L)
    bd = np.ascontiguousarray(bounds, np.int64)
    nr = C.c_int64()
    _abi.check(L.pr_aln_exchange(ctx.h, comm.h if comm is not None else None, int(s), _abi.ptr(bd, C.c_int64),
                                 C.byref(nr)), "pr_aln_exchange")
    return nr.value


def exchange_sources(ctx) -> List[int]:
    """Records the last exchange delivered to this rank, by source rank (pr_aln_exchange_sources)."""
    L = _abi.lib()
    L.pr_aln_exchange_sources.argtypes = [C.c_void_p, _abi.P64, C.c_int, _abi.P32]
    v = np.zeros(64, np.int64)
    w = C.c_int32()
    _abi.check(L.pr_aln_exchange_sources(ctx.h, _abi.ptr(v, C.c_int64), 64, C.byref(w)), "pr_aln_exchange_sources")
    return [int(x) for x in v[:w.value]]


def exchange_local(ctxs, starts, bounds: np.ndarray) -> List[int]:
    """Step 2 among several contexts of this process (pr_aln_exchange_local: the same packs,
    device copies in place of RCCL): context k holds the shard starting at starts[k]."""
    L = _abi.lib()
    _setup(L)
    w = len(ctxs)
    hs = (C.c_void_p * w)(*[c.h for c in ctxs])
    s0 = np.ascontiguousarray(starts, np.int64)
    bd = np.ascontiguousarray(bounds, np.int64)
    nr = np.zeros(w, np.int64)
    _abi.check(L.pr_aln_exchange_local(hs, w, _abi.ptr(s0, C.c_int64), _abi.ptr(bd, C.c_int64),
                                       _abi.ptr(nr, C.c_int64)), "pr_aln_exchange_local")
    return [int(x) for x in nr]


class OwnedIteration(Iteration):
    """Step 3 of the exact-parity multi-GPU layout (include/prgpu.h
    pr_aln_exchange): after shard_sw + exchange, this rank's owned long reads [lo, hi) get the
    -b/-l filter, hand-off and consensus over the alignments it received (launch(); no SW).
    The results (download, results, mask_to, stats_to, masked) are those of the owned reads
    and equal a single-GPU Iteration's on them."""

    def __init__(self, ctx, lo: int, hi: int, lr_off: np.ndarray, ref_seq: Optional[np.ndarray],
                 ref_qual: Optional[np.ndarray], sr: Optional[np.ndarray], sr_off: np.ndarray,
                 from_set: bool = False, resident_sr: bool = False):
        """lr_off: every long read's offsets; ref_seq / ref_qual: the consensus reference
        (ASCII, bam2cns --ref) and qualities of all long reads in lr_off's layout (the owned
        slice is uploaded; ref_seq None: the SW batch's long reads, when the mapping reference
        is the consensus reference); sr / sr_off: every short read of the task (nt4), which
        the consensus reads by global id (sr None: the SW batch holds every short read);
        from_set: the reference and qualities are the resident long-read set's (LongReadSet;
        ref_seq / ref_qual not used); resident_sr: the short reads are the resident ones
        (GpuStages.load_short_reads / pr_srset_load; sr must be None): read in place."""
        self.L = _abi.lib()
        _setup(self.L)
        self.ctx = ctx
        self.lo, self.hi = lo, hi
        lr_off = np.asarray(lr_off, np.int64)
        a0, a1 = int(lr_off[lo]), int(lr_off[hi])
        if (ref_seq is not None and len(ref_seq) != int(lr_off[-1])) or \
                (ref_qual is not None and len(ref_qual) != int(lr_off[-1])):
            raise ValueError("ref_seq / ref_qual must have every long read's layout (lr_off)")
        self._own_off = np.ascontiguousarray(lr_off[lo:hi + 1] - a0, np.int64)
        self._ref = None if ref_seq is None else np.ascontiguousarray(ref_seq[a0:a1], np.uint8)
        self._qual = None if ref_qual is None else np.ascontiguousarray(ref_qual[a0:a1], np.uint8)
        self._sr = None if sr is None else np.ascontiguousarray(sr, np.uint8)
        self._sr_off = np.ascontiguousarray(sr_off, np.int64)
        ob = OwnBatch()
        ob.lr0, ob.n_lr = lo, hi - lo
        ob.lr_off = _abi.ptr(self._own_off, C.c_int64)
        ob.ref_seq = _abi.ptr(self._ref, C.c_uint8)
        if self._qual is not None:
            ob.lr_qual = _abi.ptr(self._qual, C.c_uint8)
        ob.n_sr = len(self._sr_off) - 1
        ob.sr_off = _abi.ptr(self._sr_off, C.c_int64)
        ob.sr_seq = _abi.ptr(self._sr, C.c_uint8)
        ob.from_set = (1 if from_set else 0) | (2 if resident_sr else 0)   # PR_OWN_FROM_SET | PR_OWN_RESIDENT_SR
        self._ob = ob
        _abi.check(self.L.pr_iter_upload_owned(ctx.h, C.byref(ob)), "pr_iter_upload_owned")
        self.d = SimpleNamespace(lr_off=self._own_off)
        self._bounds()

    def _bounds(self):
        nl, nt, bd = C.c_int32(), C.c_int64(), _abi.CnsBounds()
        _abi.check(self.L.pr_iter_bounds(self.ctx.h, C.byref(nl), C.byref(nt), C.byref(bd)), "pr_iter_bounds")
        self.n_lr, self.n_task, self.bounds = nl.value, nt.value, bd
        self.out = None

    def launch(self, sw_opts: sw.SwOpts, params: cns.CnsParams):
        """-b/-l filter, hand-off and consensus over the alignments of the last exchange."""
        super().launch(sw_opts, params)
        self._bounds()   # the alignments are counted at launch (the output buffers follow)


class LongReadSet:
    """The resident long-read set (include/prgpu.h pr_lrset_*): the loop's current reads and
    qualities (LR.fq) and their mapping reference (LR.masked.fa) in HBM between tasks."""

    MAP, READS = 0, 1

    def __init__(self, ctx, seq_pool: np.ndarray, off: np.ndarray, qual_pool: np.ndarray):
        """ASCII bases and phred+33 qualities of every long read in one pool each (off[n+1])."""
        self.L = _abi.lib()
        _setup(self.L)
        self.ctx = ctx
        off = np.ascontiguousarray(off, np.int64)
        seq = np.ascontiguousarray(seq_pool, np.uint8)
        qual = np.ascontiguousarray(qual_pool, np.uint8)
        if len(seq) != int(off[-1]) or len(qual) != int(off[-1]):
            raise ValueError("pools must have the offsets' layout")
        _abi.check(self.L.pr_lrset_load(ctx.h, len(off) - 1, _abi.ptr(off, C.c_int64), _abi.ptr(seq, C.c_uint8),
                                        _abi.ptr(qual, C.c_uint8)), "pr_lrset_load")
        self.n = len(off) - 1

    def offsets(self) -> np.ndarray:
        off = np.zeros(self.n + 1, np.int64)
        _abi.check(self.L.pr_lrset_download(self.ctx.h, _abi.ptr(off, C.c_int64), None, None, None),
                   "pr_lrset_download")
        return off

    def download(self, seq: bool = True, qual: bool = True, mapping: bool = False):
        """-> (offsets, ASCII bases, qualities, mapping reference); pools not asked for are None."""
        off = self.offsets()
        nb = int(off[-1])
        bufs = [np.zeros(nb + 1, np.uint8) if w else None for w in (seq, qual, mapping)]
        _abi.check(self.L.pr_lrset_download(self.ctx.h, None, *[_abi.ptr(b, C.c_uint8) for b in bufs]),
                   "pr_lrset_download")
        return (off, *[None if b is None else b[:nb] for b in bufs])

    def index(self, which: int):
        """Seed index over the mapping reference (MAP) or the reads (READS), replacing the
        context's (pr_lrset_index); -> its build time (ms)."""
        from . import seed
        seed._setup(self.L)
        _abi.check(self.L.pr_lrset_index(self.ctx.h, int(which)), "pr_lrset_index")
        return seed._last_ms(self.L.pr_seed_gpu_index_last_ms, self.ctx)

    def commit(self, comm=None, with_mask: bool = False, dry: bool = False):
        """Every read's consensus (with_mask: and its masked copy as the next mapping reference)
        replaces the set's; comm: the owned batches of all ranks, all-gathered on the device.
        dry: every step of the commit without replacing the set (PR_LRSET_COMMIT_DRY)."""
        flags = (1 if with_mask else 0) | (2 if dry else 0)
        _abi.check(self.L.pr_lrset_commit(self.ctx.h, comm.h if comm is not None else None, flags),
                   "pr_lrset_commit")


class SetIteration(Iteration):
    """A world-1 iteration over the resident long-read set (pr_iter_upload_lrset): the seeds
    the last pr_seed_gpu_map left in HBM against the set's index (LongReadSet.index), the
    set's reads and qualities as the consensus reference (bam2cns --ref)."""

    def __init__(self, ctx, sr: Optional[np.ndarray], sr_off: np.ndarray, lr_off: np.ndarray):
        """sr None: the seeding's device copy of the short reads; lr_off: the set's offsets."""
        self.L = _abi.lib()
        _setup(self.L)
        self.ctx = ctx
        self._sr_off = np.ascontiguousarray(sr_off, np.int64)
        self._sr = None if sr is None else np.ascontiguousarray(sr, np.uint8)
        b = sw.SwBatch()
        b.n_sr = len(self._sr_off) - 1
        b.sr_off = _abi.ptr(self._sr_off, C.c_int64)
        b.sr_seq = _abi.ptr(self._sr, C.c_uint8)
        self._b = b
        _abi.check(self.L.pr_iter_upload_lrset(ctx.h, C.byref(b)), "pr_iter_upload_lrset")
        self.d = SimpleNamespace(lr_off=np.ascontiguousarray(lr_off, np.int64))
        nl, nt, bd = C.c_int32(), C.c_int64(), _abi.CnsBounds()
        _abi.check(self.L.pr_iter_bounds(self.ctx.h, C.byref(nl), C.byref(nt), C.byref(bd)), "pr_iter_bounds")
        self.n_lr, self.n_task, self.bounds = nl.value, nt.value, bd
        self.out = None
