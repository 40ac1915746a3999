"""proovread's sr correction loop in one process, on one GPU.

bin/proovread runs the tasks of its mode (proovread.cfg:105-127; `sr-noccs`:
read-long, bwa-sr-1 .. bwa-sr-6, bwa-sr-finish) as separate programs joined by
files.  This module runs the same loop with the reads held in memory and the
hot stages on the device:

  read-long        (proovread:1368-1524) stubby long reads dropped, upper case,
                   IUPAC -> N, natural (`byfile`) id order; the mapping reference
                   is the read itself (`.masked.fa` with --lower-case: same codes)
  bwa-sr-k         (proovread:835-869) short reads sampled with SeqChunker
                   (cov2seqchunker, proovread:2085-2102), seeded against the
                   previous iteration's masked reads (bwa-proovread mem front end,
                   seed.SeedIndex), seed extension + CIGAR + hand-off + consensus on
                   the GPU (pr_iter_*) with the previous iteration's unmasked .fq as
                   bam2cns --ref (sequence and qualities, use_ref_qual), then
                   SeqFilter --phred-mask on the GPU (pr_mask_run) -> the next
                   mapping reference and bpN/bpt for mask_shortcut_frac
                   (proovread:1700-1720, 2026-2047)
  bwa-sr-finish    (proovread:838-850, 1572-1577) 30x sampling, finish scoring,
                   unmasked reference, --no-use-ref-qual, --max-ins-length 0,
                   --detect-chimera

The device stages are behind `GpuStages` (the product; it fails loudly without
libprgpu.so and a gfx950 device).  Tests drive the same loop with the CPU oracle
chain in place of the stages (tests/loop_oracle.py) to check the GPU loop
byte-for-byte.  Deliberate scope: one GPU, the whole read set resident (at
configs[1] size ~17 GB of device buffers, far below 288 GB); bwa-proovread's
-b/-l bin filter runs on the device between the SW stage and the hand-off (A4).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import functools
import math
import time
from types import SimpleNamespace
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import control, seqchunker, tasks as T

NT4 = np.full(256, 4, np.uint8)
for _i, _c in enumerate(b"ACGT"):
    NT4[_c] = _i
    NT4[_c + 32] = _i

# proovread.cfg:119 / 125 (the sr-noccs / mr-noccs task lists) and the per-task values the
# loop reads (tasks.py restates the cfg entries)
SR_NOCCS_TASKS = T.MODE_TASKS["sr-noccs"]
MR_NOCCS_TASKS = T.MODE_TASKS["mr-noccs"]


def hcr_mask_for(task: str) -> str:
    return T.hcr_mask(task)                                 # proovread.cfg:234-242


def sr_coverage_for(task: str) -> float:
    return T.sr_coverage(task)                              # proovread.cfg:188-192


@dataclasses.dataclass
class LoopConfig:
    coverage: float = 50.0                 # --coverage (proovread.cfg:48)
    coverage_scale_factor: float = 0.75    # proovread.cfg:256
    mask_shortcut_frac: float = 0.92       # proovread.cfg:246
    mask_min_gain_frac: float = 0.03       # proovread.cfg:249
    sampling: bool = True                  # --no-sampling turns it off
    min_sr_length: Optional[int] = None    # proovread:530-532 (None: shortest short read)
    lr_min_length: Optional[int] = None    # cfg lr-min-length (None: 2 * min_sr_length)
    mode: Optional[str] = None             # sr-noccs / mr-noccs; None: by short-read length (proovread:636-642)
    tasks: Optional[Tuple[str, ...]] = None   # None: the mode's task list (proovread.cfg:105-127)
    seed_threads: int = 0
    bin_filter: bool = True                # bwa-proovread -b/-l in every iteration (proovread:1302-1313)
    exact_layout: bool = False             # world 1: run the multi-GPU exact-parity layout anyway (tests)
    keep_masked: bool = False              # LoopResult.masked: the last regular task's masked reads


class LongReads:
    """The current long-read set: the .fq of the last task (ids, sequences, qualities), held as
    byte pools with offsets (ASCII bases, phred+33 qualities); `seqs` / `quals` are per-read
    views built on first use."""

    def __init__(self, ids: List[str], seqs: Optional[List[bytes]] = None, quals: Optional[List[bytes]] = None,
                 pools: Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]] = None):
        self.ids = ids
        if pools is None:
            pools = (*_pool(seqs), _pool(quals)[0])
        self.seq_pool, self.off, self.qual_pool = pools
        self._seqs, self._quals = seqs, quals

    @property
    def seqs(self) -> List[bytes]:
        if self._seqs is None:
            self._seqs = _split(self.seq_pool, self.off)
        return self._seqs

    @property
    def quals(self) -> List[bytes]:
        if self._quals is None:
            self._quals = _split(self.qual_pool, self.off)
        return self._quals

    def pool(self, which: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
        return _pool(which)

    def fastq(self) -> str:
        return "".join(f"@{i}\n{s.decode()}\n+\n{q.decode()}\n" for i, s, q in zip(self.ids, self.seqs, self.quals))


def _pool(items: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    off = np.zeros(len(items) + 1, np.int64)
    np.cumsum([len(s) for s in items], out=off[1:])
    buf = np.frombuffer(b"".join(items), np.uint8).copy() if items else np.zeros(0, np.uint8)
    return buf, off


def _split(pool: np.ndarray, off: np.ndarray) -> List[bytes]:
    b = pool.tobytes()
    return [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]


@dataclasses.dataclass
class TaskLog:
    task: str
    n_sr: int = 0
    n_tasks: int = 0
    bpt: int = 0
    bpn: int = 0
    masked_frac: Optional[float] = None
    shortcut: str = ""
    wall_ms: Optional[float] = None        # the task's wall time in run()
    device_ms: Optional[float] = None      # kernel time the device stages report (HIP events), if any
    stage_ms: Optional[Dict[str, float]] = None   # ... per stage (index, seeding, SW, hand-off, consensus)
    part_ms: Optional[Dict[str, float]] = None    # host wall clock per part of the device task (GpuStages)
    pre_ms: Optional[float] = None         # the task's host time before the stages are called


@dataclasses.dataclass
class LoopResult:
    reads: LongReads
    chim: List[str]                        # .chim.tsv lines of the finish task (id from to score)
    ignored: List[str]                     # .ignored.tsv lines (stubby reads)
    log: List[TaskLog]
    masked: Optional[List[bytes]] = None   # the last regular iteration's masked reads (keep_masked)


# ---------------------------------------------------------------------------- read-long
_LR_TABLE = bytes(c if chr(c) in "ACGTN" else (c - 32 if chr(c) in "acgtn" else ord("N")) for c in range(256))


def read_long(records: Sequence[Tuple[str, bytes, Optional[bytes]]], stubby_length: int) -> Tuple[LongReads, List[str]]:
    """proovread:1368-1524 on (id, seq, qual or None) records: FASTA reads get '$'
    qualities, reads shorter than stubby_length go to .ignored.tsv, sequences are
    upper-cased with every non-ACGTN char -> N, ids in `byfile` order."""
    from .bam2cns import byfile_cmp
    keep: Dict[str, Tuple[bytes, bytes]] = {}
    ignored = []
    for rid, seq, qual in records:
        if len(seq) < stubby_length:
            ignored.append(f"{rid}\tstubby")
            continue
        if rid in keep:
            raise ValueError(f"Non-unique long read id ({rid})")
        s = seq.translate(_LR_TABLE)   # upper case, every non-ACGTN -> N
        keep[rid] = (s, qual if qual is not None else b"$" * len(s))
    ids = sorted(keep, key=functools.cmp_to_key(byfile_cmp))
    return LongReads(ids, [keep[i][0] for i in ids], [keep[i][1] for i in ids]), ignored


# ---------------------------------------------------------------------------- short reads
class ShortReads:
    """The short-read input as one byte stream (`cat $or_files`, proovread:1293) with its
    FASTQ/FASTA records, sampled per task like SeqChunker.  The records' sequences are kept
    as one nt4 pool in stream order; SeqChunker's chunks are contiguous record ranges, so a
    task's sample is a concatenation of pool slices."""

    def __init__(self, data: bytes, chunk_number: int = 1000):
        self.data = data
        total = len(data)
        rec = _fastq4_native(data)
        if rec is not None:   # plain 4-line FASTQ: record starts, offsets and nt4 pool in one native pass
            starts, self.off, self.pool = rec
        else:                 # FASTA (multi-line) or irregular FASTQ: the record parser
            spans = list(seqchunker.records(data))
            starts = np.array([x for x, _ in spans], np.int64)
            seqs = [self._seq_of(data[x:e]) for x, e in spans]
        self.n_chunks = max(1, chunk_number)
        csize = max(1, math.ceil(total / self.n_chunks)) if total else 1
        chunk_of = np.minimum(starts // csize, self.n_chunks - 1) if len(starts) else np.zeros(0, np.int64)
        # records of chunk k (1-based): [cfirst[k-1], cfirst[k])
        self.cfirst = np.searchsorted(chunk_of, np.arange(self.n_chunks + 1), side="left").astype(np.int64)
        if rec is None:
            self.pool, self.off = _pool(seqs)
            self.pool = NT4[self.pool]
        self.lengths = np.diff(self.off)

    @classmethod
    def from_pool(cls, pool: np.ndarray, off: np.ndarray, chunk_number: int = 1000) -> "ShortReads":
        """The reads of an nt4 pool as the FASTQ stream `@sr<i>` / sequence / `+` / quality
        records would hold them (SeqChunker chunks by byte offset), without building the bytes."""
        self = cls.__new__(cls)
        self.data = None
        off = np.ascontiguousarray(off, np.int64)
        n = len(off) - 1
        lens = np.diff(off)
        digits = np.ones(n, np.int64)
        for k in range(1, 20):
            digits += np.arange(n) >= 10 ** k
        rec = (4 + digits) + lens + 1 + 2 + lens + 1    # "@sr<i>\n" seq "\n+\n" qual "\n"
        starts = np.zeros(n, np.int64)
        if n:
            np.cumsum(rec[:-1], out=starts[1:])
        total = int(rec.sum())
        self.n_chunks = max(1, chunk_number)
        csize = max(1, math.ceil(total / self.n_chunks)) if total else 1
        chunk_of = np.minimum(starts // csize, self.n_chunks - 1)
        self.cfirst = np.searchsorted(chunk_of, np.arange(self.n_chunks + 1), side="left").astype(np.int64)
        self.pool, self.off, self.lengths = pool, off, lens
        return self

    @staticmethod
    def _seq_of(rec: bytes) -> bytes:
        if rec[:1] == b">":
            return b"".join(rec.split(b"\n")[1:]).strip()
        return rec.split(b"\n")[1].strip()

    def sample_ranges(self, sc: Optional[Dict[str, int]]) -> Tuple[np.ndarray, np.ndarray]:
        """-> (record ranges [k, 2] of the chunks SeqChunker writes for cov2seqchunker's
        parameters (None: every record), the offsets of the sampled reads)."""
        if sc is None:
            return np.array([[0, len(self.lengths)]], np.int64), self.off
        ks = np.asarray(seqchunker.select(self.n_chunks, sc["--first-chunk"], sc["--chunk-step"],
                                          sc["--chunks-per-step"]), np.int64)
        rg = np.stack([self.cfirst[ks - 1], self.cfirst[ks]], axis=1)
        rg = rg[rg[:, 1] > rg[:, 0]]
        lens = np.concatenate([self.lengths[a:b] for a, b in rg]) if len(rg) else np.zeros(0, np.int64)
        off = np.zeros(len(lens) + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        return rg, off

    def gather(self, ranges: np.ndarray) -> np.ndarray:
        """The nt4 pool of the records in `ranges` (stream order)."""
        if len(ranges) == 1 and ranges[0, 0] == 0 and ranges[0, 1] == len(self.lengths):
            return self.pool
        parts = [self.pool[self.off[a]:self.off[b]] for a, b in ranges]
        return np.concatenate(parts) if parts else np.zeros(0, np.uint8)

    def sample(self, sc: Optional[Dict[str, int]]) -> Tuple[np.ndarray, np.ndarray]:
        """nt4 pool of the records SeqChunker writes for cov2seqchunker's parameters
        (None: every record), in stream order."""
        rg, off = self.sample_ranges(sc)
        return self.gather(rg), off


def _fastq4_native(data: bytes):
    """(record starts, sequence offsets, nt4 pool) of a FASTQ stream of plain 4-line records
    (pr_fastq4_scan / pr_fastq4_fill: '@' first, '\n' last, no CR, quality lines as long as the
    sequences), or None for anything else."""
    import ctypes as C
    from . import _abi
    if not data:
        return None
    L = _abi.lib()
    L.pr_fastq4_scan.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.pr_fastq4_fill.argtypes = [C.c_char_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    n_rec, n_bases = C.c_int64(), C.c_int64()
    if L.pr_fastq4_scan(data, len(data), C.byref(n_rec), C.byref(n_bases)) != 0:
        return None
    starts = np.zeros(n_rec.value, np.int64)
    off = np.zeros(n_rec.value + 1, np.int64)
    pool = np.zeros(n_bases.value, np.uint8)
    _abi.check(L.pr_fastq4_fill(data, len(data), NT4.ctypes.data, starts.ctypes.data, off.ctypes.data, pool.ctypes.data),
               "pr_fastq4_fill")
    return starts, off, pool


# ---------------------------------------------------------------------------- device stages
@dataclasses.dataclass
class TaskOut:
    """What a task leaves on the host (the reads stay with the stages)."""
    n_tasks: int                           # seeds of this rank's short reads
    chim: List[str]                        # finish: bam2cns chimera lines of this rank's reads
    bpt: int = 0                           # regular: SeqFilter --phred-mask statistics of this
    bpn: int = 0                           # rank's reads (the loop all-reduces them)


class GpuStages:
    """The product's device stages.  The loop's state -- the current long reads, their
    qualities and the mapping reference -- stays in HBM between tasks (iteration.LongReadSet,
    pr_lrset_*); a task uploads its sampled short reads and downloads the finish task's
    chimera lines and two counters:

      index     pr_lrset_index: the seed index of the mapping reference (finish: the reads)
      seeding   pr_seed_gpu_map, seeds kept in HBM
      world 1   pr_iter_upload_lrset + pr_iter_launch: SW + -b/-l filter + hand-off + consensus
      ranks     pr_sw_upload_gpu_seeds + pr_sw_launch on the rank's short-read shard,
                pr_aln_exchange (RCCL all-to-all to the long reads' owners),
                pr_iter_upload_owned(from_set) + pr_iter_launch
      mask      pr_iter_mask (SeqFilter --phred-mask of the resident consensus) -> bpt, bpN
      commit    pr_lrset_commit: the consensus (and masked copy) replace the set's reads;
                with ranks the owned slices are all-gathered on the device."""

    def __init__(self, ctx=None):
        from . import _abi
        self.ctx = ctx or _abi.default_context()
        self.device_ms = 0.0   # kernel time of the calls so far (index, seeding, SW .. consensus)
        self.lrs = None
        self.ids: List[str] = []

    device_short_reads = True   # world 1: a task's sample is gathered on the device (pr_srset_*)
    device_short_reads_exact = True   # ... and in the exact-parity layout (pr_srset_sample)

    def snapshot(self) -> None:
        """Keep the loaded long reads on the device (pr_lrset_snapshot) for restore()."""
        from . import _abi
        L = _abi.lib()
        L.pr_lrset_snapshot.argtypes = [C.c_void_p]
        _abi.check(L.pr_lrset_snapshot(self.ctx.h), "pr_lrset_snapshot")

    def restore(self) -> None:
        """The set back to the snapshot's reads, the mapping reference to the reads
        (pr_lrset_restore): the state right after read-long, without a host round trip."""
        from . import _abi
        L = _abi.lib()
        L.pr_lrset_restore.argtypes = [C.c_void_p]
        _abi.check(L.pr_lrset_restore(self.ctx.h), "pr_lrset_restore")

    def load(self, reads: LongReads) -> None:
        from . import iteration
        self.lrs = iteration.LongReadSet(self.ctx, reads.seq_pool, reads.off, reads.qual_pool)
        self.ids = list(reads.ids)

    def load_short_reads(self, srs: "ShortReads") -> None:
        """The whole short-read input into HBM once (pr_srset_load)."""
        from . import _abi, iteration
        L = _abi.lib()
        iteration._setup(L)
        pool = np.ascontiguousarray(srs.pool, np.uint8)
        off = np.ascontiguousarray(srs.off, np.int64)
        _abi.check(L.pr_srset_load(self.ctx.h, len(off) - 1, _abi.ptr(off, C.c_int64), _abi.ptr(pool, C.c_uint8)),
                   "pr_srset_load")

    def task(self, task: str, sr: Optional[np.ndarray], sr_off: np.ndarray, params, bin_filter, comm=None,
             exact: bool = False, mask_cfg=None, sr_ranges: Optional[np.ndarray] = None, dry: bool = False) -> TaskOut:
        """One bwa-sr task on the resident set.  mask_cfg = (hcr-mask, min_sr_length) for the
        regular tasks, None for the finish task (which maps to the unmasked reads,
        proovread:838-850); exact: the multi-GPU exact-parity layout."""
        from . import _abi, exact_shard as ex, iteration, mask, seed
        L = _abi.lib()
        seed._setup(L)
        finish = mask_cfg is None
        tp = [time.perf_counter()]   # host clock at the parts' ends (last_part_ms)
        ix_ms = self.lrs.index(self.lrs.READS if finish else self.lrs.MAP)
        tp.append(time.perf_counter())
        self.device_ms += ix_ms
        seed_opts, opts = T.options(task)
        if bin_filter:
            opts.bin_size, opts.bin_length = int(bin_filter[0]), float(bin_filter[1])
        lr_off = self.lrs.offsets()
        world, rank = (comm.world, comm.rank) if comm is not None else (1, 0)
        if comm is not None and not isinstance(comm, RcclComm):
            raise TypeError("the device stages exchange over libprgpu's communicator (comm.RcclComm / LocalComm)")
        n_sr = len(sr_off) - 1
        if not exact:
            if sr is None:   # gathered from the resident short reads (load_short_reads)
                rg = np.ascontiguousarray(sr_ranges, np.int64)
                st = np.zeros(max(1, n_sr), np.int32)
                _abi.check(L.pr_seed_gpu_map_sampled(self.ctx.h, C.byref(seed_opts), _abi.ptr(rg, C.c_int64), len(rg),
                                                     _abi.ptr(st, C.c_int32)), "pr_seed_gpu_map_sampled")
            else:
                seed._map_gpu(L, self.ctx, sr, sr_off, seed_opts, False, keep_on_device=True)
            it = iteration.SetIteration(self.ctx, None, sr_off, lr_off)
            lo, hi = 0, len(lr_off) - 1
        else:
            s, e = ex.sr_range(n_sr, world, rank)
            bounds = ex.lr_bounds(lr_off, world)
            lo, hi = int(bounds[rank]), int(bounds[rank + 1])
            if sr is None:   # the resident short reads: the shard's records gathered on the device
                rg = np.ascontiguousarray(sr_ranges, np.int64).reshape(-1, 2)
                sub = np.ascontiguousarray(sample_subranges(rg, s, e), np.int64)
                st = np.zeros(max(1, e - s), np.int32)
                _abi.check(L.pr_seed_gpu_map_sampled(self.ctx.h, C.byref(seed_opts), _abi.ptr(sub, C.c_int64), len(sub),
                                                     _abi.ptr(st, C.c_int32)), "pr_seed_gpu_map_sampled")
            else:
                a0, a1 = int(sr_off[s]), int(sr_off[e])
                seed._map_gpu(L, self.ctx, sr[a0:a1], np.asarray(sr_off[s:e + 1]) - a0, seed_opts, False,
                              keep_on_device=True)
            iteration.ShardSW(self.ctx, sr, sr_off, s, e, None, lr_off, device_pools=True).launch(opts)
            iteration.exchange(self.ctx, comm, s, bounds)
            if sr is None:   # the consensus reads any short read of the sample: gathered on the device once
                _abi.check(L.pr_srset_sample(self.ctx.h, _abi.ptr(rg, C.c_int64), len(rg)), "pr_srset_sample")
                it = iteration.OwnedIteration(self.ctx, lo, hi, lr_off, None, None, None, sr_off, from_set=True,
                                              resident_sr=True)
            else:
                it = iteration.OwnedIteration(self.ctx, lo, hi, lr_off, None, None, sr if world > 1 else None, sr_off,
                                              from_set=True)
        n_tasks = seed._count(L, self.ctx)
        sd_ms = seed._last_ms(L.pr_seed_gpu_last_ms, self.ctx)
        self.device_ms += sd_ms
        tp.append(time.perf_counter())
        it.launch(opts, params)
        tp.append(time.perf_counter())
        out = TaskOut(n_tasks, [])
        if finish:
            out.chim = it.chim_lines(self.ids[lo:hi])
        else:
            if getattr(self, "_stats", None) is None:   # the {bpt, bpN} device words, kept across tasks
                self._stats = _abi.DevBuffer(self.ctx, 16)
            it.mask_to(self._stats.ptr, mask.params(mask_cfg[0], mask_cfg[1]))
            st = self._stats.download(np.int64)
            out.bpt, out.bpn = int(st[0]), int(st[1])
        tm = it.timing()
        self.device_ms += sum(tm)
        self.last_stage_ms = {k: round(v, 2) for k, v in zip(("index", "seeding", "sw_extend", "sw_global_cigar",
                                                               "exchange_handoff", "consensus"), (ix_ms, sd_ms, *tm))}
        tp.append(time.perf_counter())
        self.lrs.commit(comm if exact else None, with_mask=not finish, dry=dry)   # dry: the set stays (bench.py)
        tp.append(time.perf_counter())
        # wall clock per part (ms, device work included): index; seeding + SW + exchange; the
        # iteration launch (hand-off, consensus; waits for it); chimera lines or masking; commit
        self.last_part_ms = {k: round((b - a) * 1e3, 2) for k, a, b in
                             zip(("index", "seed_sw_exchange", "consensus_launch", "chim_or_mask", "commit"), tp, tp[1:])}
        self.last_iteration = it   # the task's consensus outputs stay readable (tests, drivers)
        return out

    def reads(self) -> LongReads:
        off, seq, qual, _ = self.lrs.download(seq=True, qual=True)
        return LongReads(self.ids, pools=(seq, off, qual))

    def masked(self) -> List[bytes]:
        """The mapping reference of the next task (LR.masked.fa)."""
        off, _, _, m = self.lrs.download(seq=False, qual=False, mapping=True)
        return _split(m, off)


def sample_subranges(ranges: np.ndarray, s: int, e: int) -> np.ndarray:
    """The record ranges of reads [s, e) of a sample made of `ranges` ([k, 2] record ranges of
    the whole short-read stream, in sample order)."""
    out = []
    at = 0
    for a, b in np.asarray(ranges, np.int64).reshape(-1, 2).tolist():
        n = b - a
        lo, hi = max(s, at), min(e, at + n)
        if hi > lo:
            out.append((a + lo - at, a + hi - at))
        at += n
    return np.array(out, np.int64).reshape(-1, 2)


def _seed_tasks(lr_map, lr_off, sr, sr_off, seed_opts, threads):
    """bwa-mode seeds of every short read on the host (pr_seed_map)."""
    from . import seed
    ix = seed.SeedIndex(lr_map, lr_off)
    try:
        return ix.map(sr, sr_off, seed_opts, threads=threads)
    finally:
        ix.close()


def _seeds_dataset(lr_map: np.ndarray, lr_off: np.ndarray, sr: np.ndarray, sr_off: np.ndarray, tasks: np.ndarray):
    """bwa mode: the seeds of every kept chain (pr_seed_map order: grouped by short read)."""
    from .sw import SwInput
    t = tasks
    d = SimpleNamespace(lr_seq=lr_map, lr_off=lr_off, sr_seq=sr, sr_off=sr_off, n_lr=len(lr_off) - 1,
                        n_sr=len(sr_off) - 1, t_sr=t["sr"].astype(np.int32), t_lr=t["lr"].astype(np.int32),
                        t_strand=t["strand"].astype(np.uint8), t_qbeg=t["qbeg"].astype(np.int32),
                        t_rbeg=t["rbeg"].astype(np.int32), t_slen=t["slen"].astype(np.int32),
                        t_chain=t["chain"].astype(np.int32))
    d.sw_input = lambda: SwInput(d.sr_off, d.sr_seq, d.lr_off, d.lr_seq, d.t_sr, d.t_lr, d.t_strand, d.t_qbeg,
                                 d.t_rbeg, d.t_slen, d.t_chain)
    return d


def _rename(lines: List[str], rid: str) -> List[str]:
    return [rid + "\t" + ln.split("\t", 1)[1] for ln in lines]


# ---------------------------------------------------------------------------- multi-rank
# The collectives of the multi-rank loop (comm.py).  Layout: SURVEY.md §8e's exact-parity
# option (exact_shard.py): every rank keeps the whole read set and the index of all long
# reads, seeds and aligns a contiguous shard of the sampled short reads (bwa mode: every
# read's alignment is decided on one rank, as bwa decides it over all long reads), sends
# each reported alignment to the owner of its long read and corrects and masks the long
# reads it owns (stages.owned_iteration; GpuStages does all of it on the device, the
# alignments crossing GPUs as one RCCL all-to-all of device buffers); the corrected and
# masked reads are then all-gathered for the next task's index and consensus reference,
# and bpt/bpN all-reduced so every rank takes the same mask_shortcut decision (the north
# star's per-iteration statistics gather).  GPU ranks use comm.RcclComm (RCCL inside
# libprgpu); the CPU tests use comm.TorchComm (gloo) with the oracle stages.
from .comm import LocalComm, LocalGroup, RcclComm, TorchComm  # noqa: E402,F401
Comm = TorchComm


# ---------------------------------------------------------------------------- the loop
def run(lr_records: Sequence[Tuple[str, bytes, Optional[bytes]]], sr_data: bytes, cfg: Optional[LoopConfig] = None,
        stages=None, comm=None) -> LoopResult:
    """The sr-noccs loop (bin/proovread:705-905) from long-read records and the short-read
    FASTQ/FASTA stream; returns the finish task's reads and chimera lines and a log per task.
    With `comm` (world > 1) every rank calls run() on the same inputs and gets the same
    result; the work is split as Comm describes.  n_tasks in the log is the rank's share."""
    cfg = cfg or LoopConfig()
    stages = stages or GpuStages()
    srs = ShortReads(sr_data)
    min_sr = cfg.min_sr_length or (int(srs.lengths.min()) if len(srs.lengths) else 200)
    stubby = cfg.lr_min_length if cfg.lr_min_length is not None else 2 * min_sr
    mode = cfg.mode or T.mode_for(min_sr)
    tasks = list(cfg.tasks or T.MODE_TASKS[mode])
    ids: List[str] = []
    ignored: List[str] = []
    log: List[TaskLog] = []
    if tasks and tasks[0] == "read-long":   # proovread:705 (the first task of every mode)
        reads, ignored = read_long(lr_records, stubby)
        ids = reads.ids
        stages.load(reads)    # the mapping reference starts as the reads (.masked.fa)
        if hasattr(stages, "load_short_reads"):
            stages.load_short_reads(srs)
        log.append(TaskLog("read-long"))
        tasks = tasks[1:]
    chim, last_masked, tlog = run_tasks(stages, srs, tasks, cfg, mode, min_sr, bool(ids), comm)
    log += tlog
    reads = stages.reads() if ids else LongReads([], [], [])
    if cfg.keep_masked and last_masked is None and ids:
        last_masked = stages.masked()
    return LoopResult(reads, chim, ignored, log, last_masked)


def run_tasks(stages, srs: ShortReads, tasks: List[str], cfg: LoopConfig, mode: str, min_sr: int, have_reads: bool,
              comm=None, sampler: Optional[control.Sampler] = None, sample_shard: Optional[Tuple[int, int]] = None,
              on_task=None) -> Tuple[List[str], Optional[List[bytes]], List[TaskLog]]:
    """The bwa-sr / bwa-mr tasks of the loop after read-long (bin/proovread:705-905) on the
    stages' resident long reads: per task SeqChunker sampling, the task on the stages, the
    {bpt, bpN} statistic (all-reduced over ranks) and mask_shortcut_frac's splice of the task
    list.  -> (chimera lines of the finish task, the masked reads kept by cfg.keep_masked or
    None, a log per task).  sample_shard (rank, world) (tests): every task sees only that
    rank's contiguous share of its sample -- one rank's seeding and SW of an N-rank run, at
    world 1; on_task(task) (tests): called before each task."""
    from . import cns
    sampler = sampler or control.Sampler(sampling=cfg.sampling)
    tasks = list(tasks)
    fracs: List[float] = []
    log: List[TaskLog] = []
    chim: List[str] = []
    last_masked = None
    tc = 0
    while tc < len(tasks):   # proovread:705 (tasks may shrink: mask_shortcut_frac splices)
        task = tasks[tc]
        if not (task.startswith("bwa-sr") or task.startswith("bwa-mr")):
            raise ValueError(f"task {task} is outside the sr / mr loops")
        finish = task.endswith("-finish")
        ent = TaskLog(task)
        t_task = time.perf_counter()
        dev0 = getattr(stages, "device_ms", None)
        task_cov = sr_coverage_for(task)
        multi = comm is not None and comm.world > 1
        ranges, sr_off = srs.sample_ranges(sampler.cov2seqchunker(cfg.coverage, task_cov))
        if sample_shard is not None:
            from .exact_shard import sr_range
            s0, s1 = sr_range(len(sr_off) - 1, sample_shard[1], sample_shard[0])
            ranges = sample_subranges(ranges, s0, s1)
            sr_off = np.ascontiguousarray(sr_off[s0:s1 + 1] - sr_off[s0], np.int64)
        if on_task is not None:
            on_task(task)
        # device stages: the sample is gathered from the resident short reads on the device
        on_dev = bool(getattr(stages, "device_short_reads", False)) and \
            (not (multi or cfg.exact_layout) or bool(getattr(stages, "device_short_reads_exact", False)))
        sr = None if on_dev else srs.gather(ranges)
        ent.n_sr = len(sr_off) - 1
        max_cov = min(cfg.coverage, task_cov) * cfg.coverage_scale_factor     # proovread:1541
        params = cns.CnsParams(coverage=max_cov, use_ref_qual=not finish, detect_chimera=finish,
                               max_ins_length=0)
        # bwa-proovread -b BIN -l BIN*min(cov, task cov) (proovread:1302-1313, cfg bin-size)
        bsz = T.bin_size(mode)
        binf = (bsz, bsz * min(cfg.coverage, task_cov)) if cfg.bin_filter else None
        if finish and cfg.keep_masked:
            last_masked = stages.masked()
        ent.pre_ms = round((time.perf_counter() - t_task) * 1e3, 2)   # (host: sampling and set-up)
        r = stages.task(task, sr, sr_off, params, binf, comm, multi or cfg.exact_layout,
                        None if finish else (hcr_mask_for(task), min_sr), sr_ranges=ranges) if have_reads \
            else TaskOut(0, [])
        ent.n_tasks = r.n_tasks
        lines, bpt, bpn = r.chim, r.bpt, r.bpn
        if multi:
            if finish:
                lines = [x.decode() for x in comm.allgather_lists([x.encode() for x in lines])]
            else:
                bpt, bpn = comm.allreduce_ints([bpt, bpn])
        chim += lines
        if not finish:
            ent.bpt, ent.bpn = bpt, bpn
            ent.masked_frac = control.masked_fraction(bpt, bpn) if bpt else 0.0
            ent.shortcut = control.mask_shortcut(tasks, tc, ent.masked_frac, fracs, cfg.mask_shortcut_frac,
                                                 cfg.mask_min_gain_frac)
        ent.wall_ms = round((time.perf_counter() - t_task) * 1e3, 1)
        if dev0 is not None:
            ent.device_ms = round(stages.device_ms - dev0, 1)
            ent.stage_ms = getattr(stages, "last_stage_ms", None)
            ent.part_ms = getattr(stages, "last_part_ms", None)
        log.append(ent)
        tc += 1
    return chim, last_masked, log


# ---------------------------------------------------------------------------- outputs
def write_outputs(res: LoopResult, pre: str, min_length: int = 500, trim_win: str = "12,5") -> None:
    """The files of bin/proovread:905-958 (without siamaera, which needs BLAST):
    PRE.untrimmed.fq, PRE.chim.tsv (ChimeraToSeqFilter of the finish task's chimera lines),
    PRE.trimmed.fq (SeqFilter --trim-win 12,5 --min-length 500 --substr PRE.chim.tsv,
    proovread.cfg:152-155) and PRE.trimmed.fa; also PRE.ignored.tsv."""
    import os
    from . import chimera_filter, seqfilter
    with open(pre + ".untrimmed.fq", "w") as f:
        f.write(res.reads.fastq())
    raw = ["#id\tfrom\tto\tscore"] + res.chim          # correct_sr_mt's header (proovread:1679)
    with open(pre + ".chim.tsv", "w") as f:
        f.write("".join(x + "\n" for x in chimera_filter.convert(raw)))
    with open(pre + ".ignored.tsv", "w") as f:
        f.write("".join(ln + "\n" for ln in res.ignored))
    rc = seqfilter.run(["--trim-win", trim_win, "--min-length", str(min_length), "--substr", pre + ".chim.tsv",
                        "--in", pre + ".untrimmed.fq", "--out", pre + ".trimmed.fq", "--phred-offset", "33"])
    if rc:
        raise RuntimeError("SeqFilter trimming failed")
    if os.path.getsize(pre + ".trimmed.fq"):   # proovread:947
        seqfilter.run(["--in", pre + ".trimmed.fq", "--out", pre + ".trimmed.fa", "--fasta", "--phred-offset", "33"])


# ---------------------------------------------------------------------------- command line
def main(argv: Optional[Sequence[str]] = None) -> int:
    """python -m proovread_amd.correct -l LR.fq -s SR.fq [-s ...] --pre OUT [--coverage C]

    Writes write_outputs' files (OUT.untrimmed.fq, OUT.trimmed.fq/.fa, OUT.chim.tsv,
    OUT.ignored.tsv).
    Launched with torch.distributed.run (one rank per GPU), the ranks split the work as
    Comm describes and rank 0 writes the files."""
    import argparse
    import os
    import sys
    from .bwa_proovread import read_fastx
    ap = argparse.ArgumentParser(prog="proovread_amd.correct")
    ap.add_argument("-l", "--long-reads", action="append", required=True)
    ap.add_argument("-s", "--short-reads", action="append", required=True)
    ap.add_argument("-p", "--pre", required=True)
    ap.add_argument("--coverage", type=float, default=50.0)
    ap.add_argument("--no-sampling", action="store_true")
    ap.add_argument("-t", "--threads", type=int, default=0)
    a = ap.parse_args(argv)
    lrs = []
    for f in a.long_reads:
        names, seqs, quals = read_fastx(f)
        lrs += list(zip(names, seqs, quals))
    sr_data = b"".join(open(f, "rb").read() for f in a.short_reads)
    cfg = LoopConfig(coverage=a.coverage, sampling=not a.no_sampling, seed_threads=a.threads)
    comm, rank = None, 0
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from . import _abi
        ctx = _abi.Context(int(os.environ.get("LOCAL_RANK", "0")))
        comm = RcclComm.from_env(ctx)   # RCCL inside libprgpu: no second HIP runtime in the process
        rank = comm.rank
        stages = GpuStages(ctx)
    else:
        stages = GpuStages()
    res = run(lrs, sr_data, cfg, stages=stages, comm=comm)
    if rank == 0:
        write_outputs(res, a.pre)
        for e in res.log:
            if e.masked_frac is not None:
                print(f"{e.task}: {e.n_sr} short reads, masked {100 * e.masked_frac:.1f}% {e.shortcut}", file=sys.stderr)
    if comm is not None:
        comm.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
