"""`bwa-proovread`-compatible mapper: the SW-stage drop-in of SURVEY.md §8(b).

proovread calls (bin/proovread:1270, 1313; options from proovread.cfg:318-333):

    bwa-proovread index REF PREFIX
    bwa-proovread mem -b BIN -l LEN -a -Y -A 5 -B 11 -O 2,1 -E 4,3 -T 2.5 \\
        -k 12 -W 20 -w 40 -r 1 -D 0 -y 20 -L 30,30 [-t N] REF /dev/fd/0 > SAM

`index` checks the long-read file and records it (the seed index is rebuilt in
memory by `mem`, in about a second per 15 Mb).  `mem` reads the long reads
(FASTA/FASTQ), the short reads (FASTA/FASTQ, a file, `-` or /dev/fd/0), builds the
seed index in HBM and seeds and chains them on the GPU (pr_seed_gpu_index_build /
pr_seed_gpu_map, restating bwa's mem_collect_intv / mem_chain / mem_chain_flt), runs
bwa mode's seed extension + CIGAR on the seeds left in HBM (pr_sw_upload_gpu_seeds +
pr_sw_launch: ksw_extend2 / ksw_global2 / mem_reg2aln, bit-exact to the SW oracle),
applies -b/-l on the device (pr_sw_binfilter) and prints SAM formatted in native code
(pr_sw_sam): `QNAME FLAG RNAME POS MAPQ CIGAR * 0 0 SEQ QUAL
AS:i:score` for every chain whose alignment passes -T (AS >= T * aligned query
length, cfg:324 "per-base-score"), with SEQ/QUAL printed for secondary hits too
(bam2cns:347 needs them).  Per read the best AS is primary (MAPQ 60), others
secondary (flag 0x100, MAPQ 0).  Logs go to stderr; errors exit 1 (proovread
prints the log, proovread:1320).

`-b BIN -l LEN` (proovread:1302-1313: BIN = bin-size, LEN = BIN x min(coverage,
task coverage)) is bwa-proovread's proovread.[ch] bin filter, "reporting of
alignments is determined by score-comparison within bins" (README.org:228-236).
Its source is absent; it is restated here as the binning proovread itself uses
(Sam::Seq add_aln_by_score, Seq.pm:582-614, the B4 row of the consensus engine):
per long read, bin = int((POS + length/2) / BIN) with Sam::Alignment's length
rule (Alignment.pm:417-431), ncscore = AS/length * length/(40+length); a bin
holding more than LEN bases admits a record only if it beats the bin's lowest
ncscore, which it then evicts.  Records pass through it in output order and the
survivors are printed in that order (parity unpinned).  The rest of bwa
mem's per-read alignment (mem_chain2aln over every seed of the kept chains,
mem_sort_dedup_patch with mem_patch_reg, mem_mark_primary_se, mem_reg2sam's -T / -D
filters) runs on the device (sw.run in bwa mode).  Not restated: bwa's MAPQ model
(MAPQ is 60 for primary, 0 for secondary records).
"""
from __future__ import annotations

import argparse
import ctypes as C
import re
import gzip
import os
import sys
import time
from typing import Callable, List, Optional, Tuple

import numpy as np

from . import seed, sw

_ASCII = np.frombuffer(b"ACGTN", np.uint8)


def read_fastx(path: str) -> Tuple[List[str], List[bytes], List[Optional[bytes]]]:
    """FASTA/FASTQ (optionally gzipped) -> names (first word), sequences, qualities (None for FASTA)."""
    if path in ("-", "/dev/fd/0", "/dev/stdin"):
        fh = sys.stdin.buffer
    elif path.endswith(".gz"):
        fh = gzip.open(path, "rb")
    else:
        fh = open(path, "rb")
    names, seqs, quals = [], [], []
    try:
        first = fh.readline()
        while first and not first.strip():
            first = fh.readline()
        if not first:
            return names, seqs, quals
        if first.startswith(b">"):
            name, buf = first, []
            for line in fh:
                if line.startswith(b">"):
                    names.append(name[1:].split()[0].decode())
                    seqs.append(b"".join(buf))
                    quals.append(None)
                    name, buf = line, []
                else:
                    buf.append(line.strip())
            names.append(name[1:].split()[0].decode())
            seqs.append(b"".join(buf))
            quals.append(None)
        elif first.startswith(b"@"):
            line = first
            while line:
                if not line.strip():
                    line = fh.readline()
                    continue
                s = fh.readline().strip()
                fh.readline()
                q = fh.readline().strip()
                names.append(line[1:].split()[0].decode())
                seqs.append(s)
                quals.append(q)
                line = fh.readline()
        else:
            raise ValueError(f"{path}: neither FASTA nor FASTQ")
    finally:
        if fh is not sys.stdin.buffer:
            fh.close()
    return names, seqs, quals


def _pool(seqs: List[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    off = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    pool = sw.NT4[np.frombuffer(b"".join(seqs), np.uint8)] if seqs else np.zeros(0, np.uint8)
    return np.ascontiguousarray(pool, np.uint8), off


def _pair(s: str, cast=int) -> Tuple:
    v = [cast(x) for x in s.split(",")]
    return (v[0], v[1] if len(v) > 1 else v[0])


def parse_mem(argv: List[str]):
    ap = argparse.ArgumentParser(prog="bwa-proovread mem", add_help=False)
    ap.add_argument("-b", type=int, default=0)
    ap.add_argument("-l", type=float, default=0)
    ap.add_argument("-a", action="store_true")
    ap.add_argument("-Y", action="store_true")
    ap.add_argument("-e", action="store_true")
    ap.add_argument("-A", type=int, default=1)
    ap.add_argument("-B", type=int, default=4)
    ap.add_argument("-O", default="6,6")
    ap.add_argument("-E", default="1,1")
    ap.add_argument("-L", default="5,5")
    ap.add_argument("-T", type=float, default=30)
    ap.add_argument("-k", type=int, default=19)
    ap.add_argument("-W", type=int, default=0)
    ap.add_argument("-w", type=int, default=100)
    ap.add_argument("-r", type=float, default=1.5)
    ap.add_argument("-D", type=float, default=0.5)
    ap.add_argument("-y", type=int, default=20)
    ap.add_argument("-c", type=int, default=500)
    ap.add_argument("-d", type=int, default=100)
    ap.add_argument("-t", type=int, default=1)
    ap.add_argument("ref")
    ap.add_argument("reads")
    return ap.parse_args(argv)


def options(a) -> Tuple[seed.SeedOpts, sw.SwOpts]:
    so = seed.default_opts(False)
    so.min_seed_len, so.w, so.split_factor, so.max_mem_intv = a.k, a.w, a.r, a.y
    so.max_occ, so.drop_ratio = a.c, a.D
    # bwa: -W defaults to the minimum seed length
    so.min_chain_weight = a.W if a.W > 0 else a.k
    o_del, o_ins = _pair(a.O)
    e_del, e_ins = _pair(a.E)
    so.a, so.o_del, so.e_del, so.o_ins, so.e_ins, so.b = a.A, o_del, e_del, o_ins, e_ins, a.B
    wo = sw.default_opts(False)
    wo.a, wo.b, wo.o_del, wo.e_del, wo.o_ins, wo.e_ins = a.A, a.B, o_del, e_del, o_ins, e_ins
    wo.w, wo.zdrop = a.w, a.d
    wo.pen_clip5, wo.pen_clip3 = _pair(a.L)
    wo.min_score_per_base = a.T
    wo.drop_ratio = a.D   # mem_reg2sam drops secondaries below -D x their primary
    return so, wo


SwRunner = Callable[[sw.SwInput, sw.SwOpts], "sw.SwResult"]


def aln_length(cigar: str, seq_len: int) -> int:
    """Sam::Alignment::length (Alignment.pm:417-431): M+D if SEQ is '*' or the CIGAR starts
    or ends with S, else the SEQ length."""
    ops = [(int(n), o) for n, o in re.findall(r"(\d+)([MIDNSHP=X])", cigar)]
    if seq_len == 0 or (ops and (ops[0][1] == "S" or ops[-1][1] == "S")):
        return sum(n for n, o in ops if o in "MD")
    return seq_len


class BinFilter:
    """-b/-l score binning over the records of one run (see the module docstring)."""

    def __init__(self, bin_size: int, bin_bases: float):
        self.b, self.cap = float(bin_size), float(bin_bases)
        self.bins = {}     # (lr, bin) -> [bases, [(ncscore, rid)] descending, stable]
        self.alive = []

    def add(self, lr: int, pos1: int, length: int, score: float) -> int:
        rid = len(self.alive)
        self.alive.append(False)
        if length <= 0:
            return rid
        nc = (score / length) * (length / (40 + length))
        key = (lr, int((pos1 + length / 2.0) / self.b))
        ent = self.bins.setdefault(key, [0, []])
        lst = ent[1]
        if ent[0] > self.cap:
            if nc <= lst[-1][0]:
                return rid
            _, old, olen = lst.pop()
            self.alive[old] = False
            ent[0] -= olen
        ent[0] += length
        i = len(lst) - 1
        while i >= 0 and nc > lst[i][0]:
            i -= 1
        lst.insert(i + 1, (nc, rid, length))
        self.alive[rid] = True
        return rid


class SamIn(C.Structure):
    _fields_ = [("sr_off", C.c_void_p), ("sr_text", C.c_void_p), ("sr_qual", C.c_void_p), ("sr_names", C.c_void_p),
                ("sr_name_off", C.c_void_p), ("lr_names", C.c_void_p), ("lr_name_off", C.c_void_p),
                ("keep", C.c_void_p), ("n_threads", C.c_int32)]


def _name_pool(names: List[str]) -> Tuple[np.ndarray, np.ndarray]:
    enc = [n.encode() for n in names]
    off = np.zeros(len(enc) + 1, np.int64)
    np.cumsum([len(x) for x in enc], out=off[1:])
    return np.frombuffer(b"".join(enc) + b"\0", np.uint8).copy(), off


def _header(out, lr_names, lr_seqs, argv) -> None:
    out.write("@HD\tVN:1.5\tSO:unsorted\n")
    for n, s in zip(lr_names, lr_seqs):
        out.write(f"@SQ\tSN:{n}\tLN:{len(s)}\n")
    out.write("@PG\tID:bwa-proovread\tPN:bwa-proovread\tVN:prgpu\tCL:bwa-proovread mem " + " ".join(argv) + "\n")


def _mem_gpu(a, so, wo, argv, lr_names, lr_seqs, sr_names, sr_seqs, sr_quals, lr_pool, lr_off, sr_pool, sr_off, out,
             log, ctx=None) -> int:
    """The product path: the seed index built in HBM (pr_seed_gpu_index_build), the seeds kept
    there (pr_seed_gpu_map), bwa mode on them (pr_sw_upload_gpu_seeds + pr_sw_launch), the
    -b/-l filter on the device (pr_sw_binfilter) and the SAM text formatted natively
    (pr_sw_sam): nothing per record in Python."""
    from . import _abi, iteration
    t0 = time.perf_counter()
    ctx = ctx or _abi.default_context()
    L = _abi.lib()
    seed._setup(L)
    iteration._setup(L)
    L.pr_sw_binfilter.argtypes = [C.c_void_p, C.c_int32, C.c_double, C.c_void_p]
    L.pr_sw_sam.argtypes = [C.c_void_p, C.POINTER(SamIn), C.POINTER(C.c_void_p), C.POINTER(C.c_int64),
                            C.POINTER(C.c_int64)]
    L.pr_buffer_free.argtypes = [C.c_void_p]
    L.pr_buffer_free.restype = None
    n_lr, n_sr = len(lr_seqs), len(sr_seqs)
    _abi.check(L.pr_seed_gpu_index_build(ctx.h, lr_pool.ctypes.data, lr_off.ctypes.data, n_lr),
               "pr_seed_gpu_index_build")
    st = np.zeros(max(1, n_sr), np.int32)
    _abi.check(L.pr_seed_gpu_map(ctx.h, C.byref(so), sr_pool.ctypes.data, sr_off.ctypes.data, n_sr, None,
                                 st.ctypes.data), "pr_seed_gpu_map")
    n_seeds = C.c_int64()
    _abi.check(L.pr_seed_gpu_seed_count(ctx.h, C.byref(n_seeds)), "pr_seed_gpu_seed_count")
    print(f"[bwa-proovread] {n_sr} reads, {n_lr} long reads, {n_seeds.value} seeds (GPU)", file=log)
    iteration.ShardSW(ctx, None, sr_off, 0, n_sr, None, lr_off, device_pools=True).launch(wo)
    n_aln = C.c_int64()
    _abi.check(L.pr_sw_aln_count(ctx.h, C.byref(n_aln)), "pr_sw_aln_count")
    keep = None
    if a.b > 0 and a.l > 0:
        keep = np.zeros(max(1, n_aln.value), np.uint8)
        _abi.check(L.pr_sw_binfilter(ctx.h, int(a.b), float(a.l), keep.ctypes.data), "pr_sw_binfilter")
    text = np.frombuffer(b"".join(sr_seqs) + b"\0", np.uint8)
    quals = None
    if sr_quals and all(q is not None for q in sr_quals):
        quals = np.frombuffer(b"".join(sr_quals) + b"\0", np.uint8)
        if len(quals) != len(text):
            raise ValueError("quality lines differ in length from their sequences")
    srn, srn_off = _name_pool(sr_names)
    lrn, lrn_off = _name_pool(lr_names)
    si = SamIn(sr_off.ctypes.data, text.ctypes.data, None if quals is None else quals.ctypes.data, srn.ctypes.data,
               srn_off.ctypes.data, lrn.ctypes.data, lrn_off.ctypes.data, None if keep is None else keep.ctypes.data,
               int(a.t) if a.t and a.t > 1 else 0)
    t1 = time.perf_counter()
    buf, ln, nrec = C.c_void_p(), C.c_int64(), C.c_int64()
    _abi.check(L.pr_sw_sam(ctx.h, C.byref(si), C.byref(buf), C.byref(ln), C.byref(nrec)), "pr_sw_sam")
    t2 = time.perf_counter()
    try:
        _header(out, lr_names, lr_seqs, argv)
        # a view of the native buffer (ctypes.string_at takes a C int size: SAM text passes 2 GiB)
        data = memoryview((C.c_ubyte * ln.value).from_address(buf.value)) if ln.value else memoryview(b"")
        if hasattr(out, "buffer"):
            out.flush()
            out.buffer.write(data)
            out.buffer.flush()
        else:
            out.write(bytes(data).decode())
        del data
    finally:
        if buf.value:
            L.pr_buffer_free(buf)
    if keep is not None:
        print(f"[bwa-proovread] -b {a.b} -l {a.l}: {nrec.value} of {int(n_aln.value)} alignments kept (device filter)",
              file=log)
    print(f"[bwa-proovread] device stages {t1 - t0:.3f} s, SAM formatting {t2 - t1:.3f} s ({ln.value} bytes), "
          f"write {time.perf_counter() - t2:.3f} s", file=log)
    return 0


def mem(argv: List[str], out=None, sw_runner: Optional[SwRunner] = None, log=None, ctx=None) -> int:
    """bwa-proovread mem.  Product path: seeding, SW, -b/-l and SAM on the device and in native
    code (_mem_gpu).  sw_runner (tests): the host seeding front end (pr_seed_map) with that SW
    runner in place of the device, records formatted here."""
    out = out or sys.stdout
    log = log or sys.stderr
    a = parse_mem(argv)
    so, wo = options(a)
    t0 = time.perf_counter()
    lr_names, lr_seqs, _ = read_fastx(a.ref)
    sr_names, sr_seqs, sr_quals = read_fastx(a.reads)
    lr_pool, lr_off = _pool(lr_seqs)
    sr_pool, sr_off = _pool(sr_seqs)
    if sw_runner is None:
        print(f"[bwa-proovread] inputs read in {time.perf_counter() - t0:.3f} s", file=log)
        return _mem_gpu(a, so, wo, argv, lr_names, lr_seqs, sr_names, sr_seqs, sr_quals, lr_pool, lr_off, sr_pool,
                        sr_off, out, log, ctx)
    ix = seed.SeedIndex(lr_pool, lr_off)
    tasks = ix.map(sr_pool, sr_off, so, threads=a.t)
    ix.close()
    print(f"[bwa-proovread] {len(sr_seqs)} reads, {len(lr_seqs)} long reads, {len(tasks)} seeds", file=log)
    # bwa mode: every seed of the kept chains goes to the device, which runs mem_chain2aln,
    # mem_sort_dedup_patch, mem_mark_primary_se and mem_reg2sam's filters; the alignments come
    # back in SAM order, read by read
    inp = sw.SwInput(sr_off, sr_pool, lr_off, lr_pool, tasks["sr"].astype(np.int32), tasks["lr"].astype(np.int32),
                     tasks["strand"].astype(np.uint8), tasks["qbeg"].astype(np.int32),
                     tasks["rbeg"].astype(np.int32), tasks["slen"].astype(np.int32),
                     tasks["chain"].astype(np.int32))
    res = sw_runner(inp, wo)
    _header(out, lr_names, lr_seqs, argv)
    filt = BinFilter(a.b, a.l) if a.b > 0 and a.l > 0 else None
    records = []
    for i in range(res.n):
        if res["status"][i] != 0 or not res["pass"][i]:
            continue
        x = int(res["task"][i])
        r, lr, strand = int(tasks["sr"][x]), int(tasks["lr"][x]), int(tasks["strand"][x])
        q = sr_seqs[r]
        qual = sr_quals[r]
        if strand:
            codes = sw.NT4[np.frombuffer(q, np.uint8)]
            seqs = _ASCII[np.where(codes < 4, 3 - codes, 4)][::-1].tobytes().decode()
            quals = qual[::-1].decode() if qual is not None else "*"
        else:
            seqs = q.decode().upper()
            quals = qual.decode() if qual is not None else "*"
        flag = int(res["flag"][i])
        mapq = 0 if flag & 0x100 else 60   # mem_approx_mapq_se is not restated
        cig = res.cigar_str(i)
        sc = int(res["score"][i])
        pos = int(res["pos"][i])
        rec = (f"{sr_names[r]}\t{flag}\t{lr_names[lr]}\t{pos + 1}\t{mapq}\t"
               f"{cig}\t*\t0\t0\t{seqs}\t{quals}\tAS:i:{sc}\n")
        if filt is not None:
            filt.add(lr, pos + 1, aln_length(cig, len(q)), float(sc))
        records.append(rec)
    if filt is not None:
        records = [rec for rec, keep in zip(records, filt.alive) if keep]
        print(f"[bwa-proovread] -b {a.b} -l {a.l}: {len(records)} of {len(filt.alive)} records kept", file=log)
    out.write("".join(records))
    return 0


def index(argv: List[str], log=None) -> int:
    log = log or sys.stderr
    if not argv:
        raise ValueError("usage: bwa-proovread index REF [PREFIX]")
    ref = argv[0]
    prefix = argv[1] if len(argv) > 1 else ref
    names, seqs, _ = read_fastx(ref)
    with open(prefix + ".prgpu", "w") as fh:
        fh.write(f"{os.path.abspath(ref)}\t{len(names)}\t{sum(len(s) for s in seqs)}\n")
    print(f"[bwa-proovread] index: {len(names)} sequences, {sum(len(s) for s in seqs)} bp (built at mem time)",
          file=log)
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in ("index", "mem"):
        print("usage: bwa-proovread index REF [PREFIX] | mem [options] REF READS", file=sys.stderr)
        return 1
    try:
        return index(argv[1:]) if argv[0] == "index" else mem(argv[1:])
    except SystemExit as e:   # argparse
        return 1 if e.code else 0
    except Exception as e:   # bwa exits non-zero, proovread prints the log (proovread:1320)
        print(f"[bwa-proovread] error: {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
