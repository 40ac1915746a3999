"""ORACLE — TEST / BASELINE INFRASTRUCTURE ONLY.

CPU restatement of one proovread correction iteration, used as the checker of
the GPU pipeline and as bench.py's cpu_baseline leg (kind "port"): bwa mem's
per-read alignment over the seeds of every short read (oracle/aln_oracle.c:
mem_chain2aln over every seed with the SW oracle oracle/sw_oracle.c,
mem_sort_dedup_patch, mem_mark_primary_se, mem_reg2sam's filters and order; or,
for a single-seed task list, the SW oracle per task), SAM records with AS:i in
bwa's output order, bwa-proovread's -b/-l filter, the per-long-read coordinate
order samtools would produce, and the consensus oracle (oracle/cns_oracle.c,
restatement of bam2cns / Sam::Seq, pinned to the reference's Perl engine).
"""
from __future__ import annotations

import ctypes as C
import multiprocessing as mp
import os
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent / "tests"))
import oracle_bind as ob  # noqa: E402

_ASCII = np.frombuffer(b"ACGTN", np.uint8)
_D = None        # dataset shared with forked workers
_OPTS = None
_PARAMS = None
_REF = None      # optional ASCII consensus reference pool (lr_off layout), else the mapped reads
_QUAL = None     # optional reference qualities (phred+33), else '$'
_FULL = False    # return (rc, fastq, trace, chim) instead of (rc, fastq)
_BINF = None     # (BIN, LEN) of bwa-proovread -b/-l, or None
_AOPTS = None    # bwa mode: oracle_bind.OalnOpts
_SEEDS = None    # bwa mode: int32 [n_seed, 10] in OalnSeed layout, and per-read offsets
_SEED_FIRST = None
_RECS = None     # bwa mode: per long read, its records in bwa output order


def _aln_length(cig, lq):
    """Sam::Alignment::length (Alignment.pm:417-431): M+D when SEQ is empty or the CIGAR
    starts or ends with S, else the SEQ length."""
    ops = [(x >> 4, x & 15) for x in cig]
    if lq == 0 or (ops and (ops[0][1] == 4 or ops[-1][1] == 4)):
        return sum(n for n, o in ops if o in (0, 2))
    return lq


def _bin_filter(recs, bin_size, bin_len):
    """bwa-proovread -b/-l (bin/proovread:1302-1313; proovread.[ch] absent): proovread's own
    score binning (Sam::Seq add_aln_by_score, Seq.pm:582-614) over the long read's reported
    records in bwa output order: bin = int((POS + length/2) / BIN), ncscore =
    AS/length * length/(40+length), a bin holding more than LEN bases admits a record only
    if it beats the lowest ncscore, which it evicts.  recs: (pos0, score, length) in task
    order -> keep flags."""
    bins, keep = {}, [False] * len(recs)
    for i, (pos0, score, length) in enumerate(recs):
        if length <= 0:
            continue
        nc = (score / length) * (length / (40 + length))
        b = int((pos0 + 1 + length / 2.0) / bin_size)
        ent = bins.setdefault(b, [0, []])
        lst = ent[1]
        if ent[0] > bin_len:
            if nc <= lst[-1][0]:
                continue
            _, old, olen = lst.pop()
            keep[old] = False
            ent[0] -= olen
        ent[0] += length
        k = len(lst) - 1
        while k >= 0 and nc > lst[k][0]:
            k -= 1
        lst.insert(k + 1, (nc, i, length))
        keep[i] = True
    return keep


def _record(lr, strand, sid, pos, cigar, score, flag, lq):
    d = _D
    so = int(d.sr_off[sid])
    q = d.sr_seq[so:so + lq]
    seq = (_ASCII[np.where(q < 4, 3 - q, 4)][::-1] if strand else _ASCII[q]).tobytes().decode()
    cg = "".join(f"{x >> 4}{'MIDNSHP=X'[x & 15]}" for x in cigar)
    line = f"sr{sid}\t{flag}\tlr{lr}\t{pos + 1}\t60\t{cg}\t*\t0\t0\t{seq}\t*\tAS:i:{score}"
    return (pos, strand, line, score, _aln_length(list(cigar), lq))


def _sr_alignments(r: int):
    """bwa mode: the reported alignments of short read r in SAM order (aln_oracle.c):
    (lr, strand, pos, cigar ops, score, flag, qb, qe, rb, re, truesc, seed task)."""
    d = _D
    L = ob.aln_lib()
    a, b = int(_SEED_FIRST[r]), int(_SEED_FIRST[r + 1])
    if a == b:
        return []
    so = int(d.sr_off[r])
    lq = int(d.sr_off[r + 1]) - so
    qp = d.sr_seq.ctypes.data + so
    outs = (ob.OalnReg * (b - a))()
    no, ne = C.c_int(), C.c_int()
    rc = L.oaln_read(C.byref(_OPTS), C.byref(_AOPTS), qp, lq, d.lr_seq.ctypes.data, d.lr_off.ctypes.data, d.n_lr,
                     _SEEDS.ctypes.data + a * 40, b - a, r, outs, C.byref(no), C.byref(ne))
    if rc:
        raise RuntimeError(f"oaln_read failed on read {r}")
    res = ob.OswResult()
    out = []
    for k in range(no.value):
        g = outs[k]
        lr = int(g.lr)
        lo = int(d.lr_off[lr])
        Llen = int(d.lr_off[lr + 1]) - lo
        L.osw_reg2aln(C.byref(_OPTS), qp, lq, d.lr_seq.ctypes.data + lo, Llen, int(g.strand), C.byref(g.g),
                      C.byref(res))
        out.append((lr, int(g.strand), int(res.pos), list(res.cigar[:res.n_cigar]), int(res.score), int(g.flag),
                    int(g.g.qb), int(g.g.qe), int(g.g.rb), int(g.g.re), int(g.g.truesc), a + int(g.seed)))
    return out


def _sr_records(r: int):
    """bwa mode: (lr, record) pairs of short read r in SAM order."""
    lq = int(_D.sr_off[r + 1] - _D.sr_off[r])
    return [(a[0], _record(a[0], a[1], r, a[2], a[3], a[4], a[5], lq)) for a in _sr_alignments(r)]


def bwa_alignments(d, task="bwa-sr", drop_ratio=None, reads=None):
    """bwa mode (d.t_chain set): per short read its reported alignments in SAM order
    (_sr_alignments tuples), single process."""
    global _D, _OPTS, _AOPTS, _SEEDS, _SEED_FIRST
    _D = d
    _OPTS = ob.sw_opts(task) if isinstance(task, str) else ob.OswOpts(*task)
    _AOPTS = ob.aln_opts(task if isinstance(task, str) else "bwa-sr")
    if drop_ratio is not None:
        _AOPTS.drop_ratio = float(drop_ratio)
    ob.build() if not ob.LIB.exists() else None
    ob.aln_lib()
    n = len(d.t_sr)
    _SEEDS = np.zeros((n, 10), np.int32)
    for k, col in enumerate(("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen")):
        _SEEDS[:, k] = getattr(d, col)
    _SEEDS[:, 8] = d.t_chain
    _SEED_FIRST = np.searchsorted(d.t_sr, np.arange(d.n_sr + 1)).astype(np.int64)
    return [_sr_alignments(r) for r in (range(d.n_sr) if reads is None else reads)]


def _lr_task_records(lr: int):
    """Single-seed tasks: the SW oracle for all tasks of long read `lr`, in task order."""
    d = _D
    L = ob.sw_lib()
    t0, t1 = int(d._task_off[lr]), int(d._task_off[lr + 1])
    lr_ptr = d.lr_seq.ctypes.data + int(d.lr_off[lr])
    Llen = int(d.lr_off[lr + 1] - d.lr_off[lr])
    recs = []
    r = ob.OswResult()
    for t in range(t0, t1):
        sid = int(d.t_sr[t])
        so = int(d.sr_off[sid])
        lq = int(d.sr_off[sid + 1]) - so
        rc = L.osw_task(C.byref(_OPTS), C.cast(d.sr_seq.ctypes.data + so, C.POINTER(C.c_uint8)), lq,
                        C.cast(lr_ptr, C.POINTER(C.c_uint8)), Llen, int(d.t_strand[t]), int(d.t_qbeg[t]),
                        int(d.t_rbeg[t]), int(d.t_slen[t]), C.byref(r))
        if rc or not getattr(r, "pass"):
            continue
        strand = int(d.t_strand[t])
        recs.append(_record(lr, strand, sid, r.pos, r.cigar[:r.n_cigar], r.score, 16 if strand else 0, lq))
    return recs


def _lr_sam_lines(lr: int):
    """The records of long read `lr` (bwa output order) -> -b/-l filter -> coordinate order:
    the SAM lines bam2cns reads for it (bin/bam2cns:336)."""
    recs = _RECS[lr] if _RECS is not None else _lr_task_records(lr)
    recs = [(x[0], x[1], i, x[2], x[3], x[4]) for i, x in enumerate(recs)]
    if _BINF is not None:   # records in bwa's output order for this long read
        keep = _bin_filter([(x[0], float(x[4]), x[5]) for x in recs], *_BINF)
        recs = [x for x, k in zip(recs, keep) if k]
    recs.sort(key=lambda x: (x[0], x[1], x[2]))
    return [x[3] for x in recs]


def _lr_chain(lr: int):
    """The records of long read `lr` (_lr_sam_lines) -> consensus."""
    d = _D
    lines = [x.encode() for x in _lr_sam_lines(lr)]
    arr = (C.c_char_p * (len(lines) + 1))(*lines)
    a, b = int(d.lr_off[lr]), int(d.lr_off[lr + 1])
    ref = _REF[a:b].tobytes() if _REF is not None else _ASCII[d.lr_seq[a:b]].tobytes()
    qual = _QUAL[a:b].tobytes() if _QUAL is not None else b"$" * len(ref)
    name = d.lr_names[lr] if hasattr(d, "lr_names") else f"lr{lr}"
    res = ob.OcnsResult()
    rc = ob.lib().ocns_run(C.byref(_PARAMS), name.encode(), ref, qual, len(ref), arr, len(lines),
                           None, 0, C.byref(res))
    if _FULL:
        out = (rc, res.fastq.decode(), res.trace.decode(), res.chim.decode()) if rc == 0 else (rc, "", "", "")
    else:
        out = (rc, res.fastq.decode() if rc == 0 else "")
    ob.lib().ocns_free(C.byref(res))
    return out


def _init_worker():
    ob.aln_lib()


def run_sample(d, lrs, task="bwa-sr", coverage=11.25, use_ref_qual=True, workers=None, ref_seq=None,
               ref_qual=None, detect_chimera=False, full=False, bin_filter=None, drop_ratio=None, sam_only=False):
    """Run the CPU chain on long reads `lrs`; returns (wall seconds, bases, results, workers).

    d.t_chain set (bwa mode): d's tasks are every seed of the kept chains grouped by short
    read; every short read with a seed on `lrs` goes through bwa mem's per-read alignment
    (all of its seeds, so the result is exact for those long reads).  Otherwise d's tasks are
    single-seed alignments grouped by long read.
    ref_seq / ref_qual: ASCII consensus reference and its qualities in the long reads' layout
    (bam2cns --ref, the previous iteration's .fq) when it differs from the mapped reads;
    full: per read (rc, fastq, trace, chim lines) instead of (rc, fastq); bin_filter: (BIN, LEN)
    of bwa-proovread -b/-l applied to each long read's records, or None; drop_ratio: bwa -D
    (default: 0.75 for bwa-sr-finish, else 0); sam_only: per read its SAM lines in coordinate
    order (what the consensus would read) instead of the consensus."""
    global _D, _OPTS, _PARAMS, _REF, _QUAL, _FULL, _BINF, _AOPTS, _SEEDS, _SEED_FIRST, _RECS
    _D = d
    _BINF = tuple(bin_filter) if bin_filter else None
    _REF = None if ref_seq is None else np.ascontiguousarray(ref_seq, np.uint8)
    _QUAL = None if ref_qual is None else np.ascontiguousarray(ref_qual, np.uint8)
    _FULL = bool(full)
    if isinstance(task, str):
        _OPTS = ob.sw_opts(task)
        _AOPTS = ob.aln_opts(task)
    else:   # (a, b, o_del, o_ins, e_del, e_ins, w, pen_clip5, pen_clip3, zdrop, min_score_per_base)
        _OPTS = ob.OswOpts(*task)
        _AOPTS = ob.aln_opts("bwa-sr")
    if drop_ratio is not None:
        _AOPTS.drop_ratio = float(drop_ratio)
    _PARAMS = ob.OcnsParams()
    _PARAMS.max_coverage = coverage
    _PARAMS.bin_size = 20.0
    _PARAMS.trim = 1
    _PARAMS.indel_taboo_length = 7
    _PARAMS.indel_taboo = 0.1
    _PARAMS.min_aln_length = 50
    _PARAMS.max_ins_length = 0
    _PARAMS.fallback_phred = 1
    _PARAMS.phred_offset = 33
    _PARAMS.ref_phred_offset = 33
    _PARAMS.use_ref_qual = int(use_ref_qual)
    _PARAMS.qual_weighted = 0
    _PARAMS.detect_chimera = int(detect_chimera)
    _PARAMS.invert_scores = 0
    ob.build() if not ob.LIB.exists() else None
    ob.aln_lib()
    workers = workers or min(16, os.cpu_count() or 1)
    lrs = list(lrs)
    if workers > 1 and _hip_in_process():   # never fork a process that holds a HIP runtime
        return _run_in_child(d, lrs, dict(task=task, coverage=coverage, use_ref_qual=use_ref_qual, workers=workers,
                                          ref_seq=ref_seq, ref_qual=ref_qual, detect_chimera=detect_chimera,
                                          full=full, bin_filter=bin_filter, drop_ratio=drop_ratio,
                                          sam_only=sam_only))
    bases = int(sum(int(d.lr_off[i + 1] - d.lr_off[i]) for i in lrs))
    bwa = getattr(d, "t_chain", None) is not None
    _RECS = None
    if bwa:
        n = len(d.t_sr)
        _SEEDS = np.zeros((n, 10), np.int32)
        for k, col in enumerate(("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen")):
            _SEEDS[:, k] = getattr(d, col)
        _SEEDS[:, 8] = d.t_chain
        _SEEDS = np.ascontiguousarray(_SEEDS)
        _SEED_FIRST = np.searchsorted(d.t_sr, np.arange(d.n_sr + 1)).astype(np.int64)
        want = np.zeros(d.n_lr, bool)
        want[lrs] = True
        reads = np.unique(d.t_sr[want[d.t_lr]]).tolist()
    elif not hasattr(d, "_task_off"):
        d._task_off = np.zeros(d.n_lr + 1, np.int64)
        np.cumsum(np.bincount(d.t_lr, minlength=d.n_lr), out=d._task_off[1:])
    t = time.perf_counter()
    if bwa:
        if workers == 1:
            per_read = [_sr_records(r) for r in reads]
        else:
            per_read = _pool_map(_sr_records, reads, workers, 64)
        _RECS = {i: [] for i in lrs}
        for recs in per_read:   # read order, then SAM order inside a read
            for lr, rec in recs:
                if lr in _RECS:
                    _RECS[lr].append(rec)
    fn = _lr_sam_lines if sam_only else _lr_chain
    if workers == 1:
        res = [fn(i) for i in lrs]
    else:
        res = _pool_map(fn, lrs, workers, 1)
    return time.perf_counter() - t, bases, res, workers


def _pool_map(fn, items, workers: int, chunksize: int):
    """fn over items on forked workers (they inherit the module's dataset).  A worker that dies
    breaks the pool and raises here (concurrent.futures' BrokenProcessPool) instead of being
    replaced silently.  Only called in a process without a HIP runtime (run_sample)."""
    from concurrent.futures import ProcessPoolExecutor
    with ProcessPoolExecutor(workers, mp_context=mp.get_context("fork"), initializer=_init_worker) as ex:
        return list(ex.map(fn, items, chunksize=chunksize))


def _hip_in_process() -> bool:
    """Whether this process has loaded the HIP runtime (a GPU test's pytest process): forking it
    is unsafe, so the worker pool then runs in a fresh child process (_run_in_child)."""
    try:
        with open("/proc/self/maps") as f:
            return any("libamdhip64" in ln for ln in f)
    except OSError:
        return False


_DATA_KEYS = ("lr_seq", "lr_off", "sr_seq", "sr_off", "t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen",
              "t_chain")


def _run_in_child(d, lrs, kw):
    """run_sample in a fresh Python process (no HIP runtime there, so it may fork its workers):
    the dataset goes through .npy files (memory-mapped by the child), the results come back as
    JSON."""
    import json
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory(prefix="cpu_chain_") as td:
        tdp = Path(td)
        meta = {"lrs": [int(x) for x in lrs], "kw": {}, "arrays": [], "lr_names": None}
        for k in _DATA_KEYS:
            v = getattr(d, k, None)
            if v is not None:
                np.save(tdp / f"{k}.npy", np.ascontiguousarray(v))
                meta["arrays"].append(k)
        if hasattr(d, "lr_names"):
            meta["lr_names"] = list(d.lr_names)
        for k, v in kw.items():
            if isinstance(v, np.ndarray):
                np.save(tdp / f"kw_{k}.npy", np.ascontiguousarray(v))
                meta["kw"][k] = {"npy": f"kw_{k}.npy"}
            else:
                meta["kw"][k] = {"value": list(v) if isinstance(v, tuple) else v}
        (tdp / "meta.json").write_text(json.dumps(meta))
        subprocess.run([sys.executable, str(Path(__file__).resolve()), "--child", td], check=True)
        out = json.loads((tdp / "out.json").read_text())
    res = [tuple(r) if isinstance(r, list) and not kw.get("sam_only") else r for r in out["res"]]
    return out["wall"], out["bases"], res, out["workers"]


def _child_main(td: str) -> None:
    import json
    from types import SimpleNamespace
    tdp = Path(td)
    meta = json.loads((tdp / "meta.json").read_text())
    d = SimpleNamespace(**{k: np.load(tdp / f"{k}.npy", mmap_mode="r") for k in meta["arrays"]})
    d.n_lr, d.n_sr = len(d.lr_off) - 1, len(d.sr_off) - 1
    if meta["lr_names"] is not None:
        d.lr_names = meta["lr_names"]
    kw = {}
    for k, v in meta["kw"].items():
        if "npy" in v:
            kw[k] = np.load(tdp / v["npy"])
        else:
            kw[k] = tuple(v["value"]) if k in ("task", "bin_filter") and isinstance(v["value"], list) else v["value"]
    wall, bases, res, workers = run_sample(d, meta["lrs"], **kw)
    (tdp / "out.json").write_text(json.dumps({"wall": wall, "bases": bases, "res": res, "workers": workers}))


if __name__ == "__main__" and len(sys.argv) == 3 and sys.argv[1] == "--child":
    _child_main(sys.argv[2])
