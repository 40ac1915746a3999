"""`bam2cns`-compatible consensus worker running on the GPU.

Drop-in for the worker command proovread fans out with `xargs -P`
(bin/proovread:1596-1619): same options as bin/bam2cns:171-205, same output
files (`PREFIX.fq`, `PREFIX.chim.tsv`, `PREFIX.ignored.tsv`,
`PREFIX.debug.trace`), same natural read order (bam2cns:324, byfile 501-517).
The consensus of every long read of the chunk is computed in ONE launch of
libprgpu.so (pr_cns_run) instead of one Perl Sam::Seq object per read.

Alignment input: `--bam FILE` (coordinate-sorted BAM, read with a built-in
BGZF/BAM reader: samtools is not needed) or `--sam FILE` (SAM text in the same
order).  Errors exit with status 255 like Verbose->exit (Verbose.pm:454).

    python -m proovread_amd.bam2cns --bam x.bam --ref lr.fq --ref-offset 0 \\
        --max-ref-seqs 100 --coverage 11.25 --prefix out/chunk0 --append
"""
from __future__ import annotations

import argparse
import ctypes as C
import dataclasses
import functools
import glob
import gzip
import os
import re
import struct
import sys
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import bamio, cns


def _perl_split_digits(s: str) -> List[str]:
    parts = re.split(r"(\d+)", s)
    while parts and parts[-1] == "":      # Perl's split drops trailing empty fields
        parts.pop()
    return parts


def _perl_num(s: str) -> float:
    m = re.match(r"\s*([+-]?\d+(?:\.\d*)?)", s)
    return float(m.group(1)) if m else 0.0


def byfile_cmp(a: str, b: str) -> int:
    """bam2cns:501-517 `byfile`: natural order over digit / non-digit runs."""
    pa, pb = _perl_split_digits(a), _perl_split_digits(b)
    for i in range(max(len(pa), len(pb))):
        if i >= len(pa):
            return -1
        if i >= len(pb):
            return 1
        x, y = pa[i], pb[i]
        if re.search(r"\d", x):
            nx, ny = _perl_num(x), _perl_num(y)
            r = (nx > ny) - (nx < ny)
        else:
            r = (x > y) - (x < y)
        if r:
            return r
    return 0


# ---------------------------------------------------------------------------
# reference reads (Fastq::Parser / Fasta::Parser subset used by bam2cns:302-322)
def guess_phred_offset(path: str, n: int = 1000) -> Optional[int]:
    """Fastq::Parser::guess_phred_offset (Parser.pm:593-633) over the first n
    records (the reference samples n random records of files >= 10 MB)."""
    lo, hi = 255, 0
    with open(path, "rb") as fh:
        for _ in range(n):
            lines = [fh.readline() for _ in range(4)]
            if not lines[3]:
                break
            q = lines[3].rstrip(b"\n")
            if q:
                lo, hi = min(lo, min(q)), max(hi, max(q))
    if hi == 0:
        return None
    if lo >= 64 and hi <= 33 + 42:
        return None
    if lo >= 33 and hi <= 33 + 42:
        return 33
    if lo >= 64 and hi <= 64 + 42:
        return 64
    return None


def read_refs(path: str, offset: int, max_reads: int) -> Tuple[List[cns.LongRead], bool]:
    """bam2cns:300-312: seek to --ref-offset, read up to --max-ref-seqs records."""
    with open(path, "rb") as fh:
        head = fh.read(1)
        is_fastq = head == b"@"
        fh.seek(offset if offset else 0)
        out: List[cns.LongRead] = []
        if is_fastq:
            while True:
                lines = [fh.readline() for _ in range(4)]
                if not lines[3]:
                    break
                h, s, _, q = (x.decode("latin-1").rstrip("\n") for x in lines)
                parts = h[1:].split(None, 1)
                out.append(cns.LongRead(parts[0], s, q, parts[1] if len(parts) > 1 else ""))
                if max_reads and len(out) >= max_reads:
                    break
        else:
            cur = None
            seq: List[str] = []
            for raw in fh:
                line = raw.decode("latin-1").rstrip("\n")
                if line.startswith(">"):
                    if cur is not None:
                        out.append(cns.LongRead(cur[0], "".join(seq), None, cur[1]))
                        if max_reads and len(out) >= max_reads:
                            cur = None
                            break
                    parts = line[1:].split(None, 1)
                    cur = (parts[0], parts[1] if len(parts) > 1 else "")
                    seq = []
                else:
                    seq.append(line.strip())
            if cur is not None and not (max_reads and len(out) >= max_reads):
                out.append(cns.LongRead(cur[0], "".join(seq), None, cur[1]))
    return out, is_fastq


# ---------------------------------------------------------------------------
# alignments: SAM text or BAM (BGZF = concatenated gzip members)
def sam_records(path: str) -> Tuple[Dict[str, int], Iterator[cns.SamRecord]]:
    hdr: Dict[str, int] = {}
    fh = open(path, "r", encoding="latin-1")
    first = []
    for line in fh:
        if line.startswith("@"):
            m = re.match(r"@SQ\t.*SN:(\S+).*\tLN:(\d+)", line)
            if m:
                hdr[m.group(1)] = int(m.group(2))
            continue
        first.append(line)
        break

    def it():
        for line in first:
            yield cns.SamRecord.from_line(line)
        for line in fh:
            if line.strip():
                yield cns.SamRecord.from_line(line)
        fh.close()
    return hdr, it()


_SEQ_NT16 = "=ACMGRSVTWYHKDBN"
_AUX_INT = {"c": "<b", "C": "<B", "s": "<h", "S": "<H", "i": "<i", "I": "<I"}
_AUX_SIZE = {"A": 1, "c": 1, "C": 1, "s": 2, "S": 2, "i": 4, "I": 4, "f": 4}


def bam_records(path: str) -> Tuple[Dict[str, int], Iterator[cns.SamRecord]]:
    fh = gzip.open(path, "rb")
    if fh.read(4) != b"BAM\x01":
        raise ValueError(f"{path}: not a BAM file")
    l_text = struct.unpack("<i", fh.read(4))[0]
    fh.read(l_text)
    n_ref = struct.unpack("<i", fh.read(4))[0]
    names, hdr = [], {}
    for _ in range(n_ref):
        ln = struct.unpack("<i", fh.read(4))[0]
        name = fh.read(ln).rstrip(b"\0").decode()
        lr = struct.unpack("<i", fh.read(4))[0]
        names.append(name)
        hdr[name] = lr

    def it():
        while True:
            b = fh.read(4)
            if len(b) < 4:
                break
            bs = struct.unpack("<i", b)[0]
            r = fh.read(bs)
            ref_id, pos, l_rn, _mapq, _bin, n_cig, _flag, l_seq = struct.unpack("<iiBBHHHi", r[:20])
            o = 32
            o += l_rn
            cig = list(struct.unpack(f"<{n_cig}I", r[o:o + 4 * n_cig]))
            o += 4 * n_cig
            sb = r[o:o + (l_seq + 1) // 2]
            o += (l_seq + 1) // 2
            seq = "".join(_SEQ_NT16[(sb[i >> 1] >> (4 * (1 - (i & 1)))) & 15] for i in range(l_seq))
            qb = r[o:o + l_seq]
            o += l_seq
            qual = "*" if (l_seq and qb[0] == 0xFF) else "".join(chr(x + 33) for x in qb)
            score = None
            while o < len(r):
                tag = r[o:o + 2].decode()
                t = chr(r[o + 2])
                o += 3
                if t in _AUX_INT:
                    v = struct.unpack(_AUX_INT[t], r[o:o + _AUX_SIZE[t]])[0]
                    o += _AUX_SIZE[t]
                    if tag == "AS":
                        score = float(v)
                elif t in ("A", "f"):
                    if tag == "AS" and t == "f":
                        score = struct.unpack("<f", r[o:o + 4])[0]
                    o += _AUX_SIZE[t]
                elif t in ("Z", "H"):
                    e = r.index(b"\0", o)
                    if tag == "AS":
                        score = cns.parse_perl_number(r[o:e].decode())
                    o = e + 1
                elif t == "B":
                    st = chr(r[o])
                    cnt = struct.unpack("<i", r[o + 1:o + 5])[0]
                    o += 5 + cnt * _AUX_SIZE[st]
                else:
                    raise ValueError(f"bad BAM aux type {t}")
            if ref_id < 0:
                continue
            yield cns.SamRecord(names[ref_id], pos + 1, cig, seq if l_seq else "*", qual, score)
        fh.close()
    return hdr, it()


class _BamAlns(C.Structure):
    _fields_ = [("n", C.c_int64), ("rid", C.c_void_p), ("pos1", C.c_void_p), ("score", C.c_void_p),
                ("flags", C.c_void_p), ("seq_off", C.c_void_p), ("lseq", C.c_void_p), ("cig_off", C.c_void_p),
                ("ncig", C.c_void_p), ("seq", C.c_void_p), ("qual", C.c_void_p), ("cig", C.c_void_p),
                ("seq_len", C.c_int64), ("cig_len", C.c_int64)]


def bam_alns_native(path: str, threads: int = 0) -> Tuple[List[str], Dict[str, np.ndarray]]:
    """Every record of a BAM decoded by libprgpu (pr_bgzf_decompress + pr_bam_decode_alns):
    reference names and the pr_cns_batch alignment columns (rid, pos1, score, flags, seq_off,
    lseq, cig_off, ncig) with their pools (seq, qual, cig) — what bam_records yields, as arrays."""
    from . import _abi
    L, _, _ = bamio._codec()
    if not getattr(L, "_bam_alns_ready", False):
        L.pr_bam_decode_alns.argtypes = [C.c_char_p, C.c_int64, C.c_int, C.POINTER(_BamAlns)]
        L.pr_bam_alns_free.argtypes = [C.POINTER(_BamAlns)]
        L.pr_bam_alns_free.restype = None
        L._bam_alns_ready = True
    with open(path, "rb") as fh:
        stream = bamio._native_inflate(fh.read(), threads)
    h, o = bamio._parse_header(stream)
    body = stream[o:]
    a = _BamAlns()
    _abi.check(L.pr_bam_decode_alns(body, len(body), threads, C.byref(a)), "pr_bam_decode_alns")
    try:
        n = a.n
        def take(ptr, ct, cnt):
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(max(cnt, 1),))[:cnt].copy()
        cols = {"rid": take(a.rid, C.c_int32, n), "pos1": take(a.pos1, C.c_int32, n),
                "score": take(a.score, C.c_double, n), "flags": take(a.flags, C.c_uint8, n),
                "seq_off": take(a.seq_off, C.c_int64, n), "lseq": take(a.lseq, C.c_int32, n),
                "cig_off": take(a.cig_off, C.c_int64, n), "ncig": take(a.ncig, C.c_int32, n),
                "seq": take(a.seq, C.c_uint8, a.seq_len), "qual": take(a.qual, C.c_uint8, a.seq_len),
                "cig": take(a.cig, C.c_uint32, a.cig_len)}
    finally:
        L.pr_bam_alns_free(C.byref(a))
    return [nm for nm, _ in h.refs], cols


def pack_bam_chunk(reads: Sequence[cns.LongRead], names: Sequence[str], A: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """pr_cns_batch for a chunk from natively decoded BAM columns: each read gets the records
    whose RNAME is its id, in file order (a repeated id gets the same records, samtools view
    "id:"); the pools stay as decoded, the columns point into them."""
    want: Dict[str, int] = {}
    for i, r in enumerate(reads):
        want.setdefault(r.id, i)
    lut = np.array([want.get(nm, -1) for nm in names] + [-1], np.int64)
    rid = A["rid"]
    if len(rid) and (rid.min() < -1 or rid.max() >= len(names)):
        die(f"BAM record with reference id outside [-1, {len(names)})")
    ridx = lut[rid] if len(rid) else np.zeros(0, np.int64)   # rid -1 -> lut[-1] = -1
    sel = np.nonzero(ridx >= 0)[0]
    if (A["flags"][sel] & _abi_flag("PR_ALN_NO_SEQ")).any():
        die("Cannot handle BAM secondary alignments without seq/qual")
    order = sel[np.argsort(ridx[sel], kind="stable")]
    counts = np.bincount(ridx[sel], minlength=len(reads))
    start = np.zeros(len(reads) + 1, np.int64)
    np.cumsum(counts, out=start[1:])
    canon = [want[r.id] for r in reads]
    if all(c == i for i, c in enumerate(canon)):
        idx = order
    else:
        idx = np.concatenate([order[start[c]:start[c + 1]] for c in canon] or [np.zeros(0, np.int64)])
    d = cns.pack_reads(reads)
    aln_off = np.zeros(len(reads) + 1, np.int64)
    np.cumsum([counts[c] for c in canon], out=aln_off[1:])
    d.update(aln_off=aln_off, aln_pos=A["pos1"][idx], aln_score=A["score"][idx], aln_flags=A["flags"][idx],
             aln_seq_off=A["seq_off"][idx], aln_lseq=A["lseq"][idx], aln_cig_off=A["cig_off"][idx],
             aln_ncig=A["ncig"][idx])
    d["seq_pool"] = A["seq"] if len(A["seq"]) else np.zeros(1, np.uint8)
    d["qual_pool"] = A["qual"] if len(A["qual"]) else np.zeros(1, np.uint8)
    d["cig_pool"] = A["cig"] if len(A["cig"]) else np.zeros(1, np.uint32)
    d["_seq_pool_len"] = np.array([len(A["seq"])], np.int64)
    d["_cig_pool_len"] = np.array([len(A["cig"])], np.int64)
    return d


def _abi_flag(name: str) -> int:
    from . import _abi
    return getattr(_abi, name)


# ---------------------------------------------------------------------------
def parse_args(argv):
    ap = argparse.ArgumentParser(prog="bam2cns", allow_abbrev=False)
    ap.add_argument("--cfg", "-c")
    ap.add_argument("--prefix", default="")
    ap.add_argument("--bam")
    ap.add_argument("--sam")
    ap.add_argument("--ref")
    ap.add_argument("--ref-offset", type=int, default=0)
    ap.add_argument("--max-ref-seqs", "--max-reads", default="0")
    ap.add_argument("--coverage", default="50")
    ap.add_argument("--qv-offset", default="33")
    ap.add_argument("--ignore-mcr", "--ignore-hcr", action="store_true")
    ap.add_argument("--use-ref-qual", dest="use_ref_qual", action="store_true", default=True)
    ap.add_argument("--no-use-ref-qual", dest="use_ref_qual", action="store_false")
    ap.add_argument("--qual-weighted", dest="qual_weighted", action="store_true", default=False)
    ap.add_argument("--no-qual-weighted", dest="qual_weighted", action="store_false")
    ap.add_argument("--detect-chimera", dest="detect_chimera", action="store_true", default=False)
    ap.add_argument("--no-detect-chimera", dest="detect_chimera", action="store_false")
    ap.add_argument("--chimera-min-score", type=float, default=0)
    ap.add_argument("--max-ins-length", type=int, default=0)
    # bam2cns:186 declares 'bin-size' without '=': it takes no value and the bin
    # size stays 20; a following number is left in @ARGV (ignored here too)
    ap.add_argument("--bin-size", action="store_true")
    ap.add_argument("--fallback-phred", type=int)
    ap.add_argument("--invert-scores", dest="invert_scores", action="store_true", default=False)
    ap.add_argument("--no-invert-scores", dest="invert_scores", action="store_false")
    ap.add_argument("--utg-mode", action="store_true")
    ap.add_argument("--rep-coverage", type=int)
    ap.add_argument("--min-ncscore", type=float)
    ap.add_argument("--haplo-coverage", action="store_true")
    ap.add_argument("--mask-weak-reads", type=int, default=20)
    ap.add_argument("--ignore-weak-reads", type=int, default=20)
    ap.add_argument("--append", dest="append", action="store_true", default=False)
    ap.add_argument("--no-append", dest="append", action="store_false")
    ap.add_argument("--samtools-path", action="store_true")
    ap.add_argument("--debug", dest="debug", action="store_true", default=False)
    ap.add_argument("--no-debug", dest="debug", action="store_false")
    ap.add_argument("--sr-min-length", action="store_true")
    args, _rest = ap.parse_known_args(argv)
    return args


_CFG_KEYS = ("sr-trim", "sr-indel-taboo-length", "sr-indel-taboo", "debug")


def read_cfg(path: str) -> Dict[str, float]:
    """The numeric Sam::Seq settings of a proovread.cfg (bam2cns:59-67 merges the
    core file and --cfg with `do FILE`).  The file is Perl; only `'key' => NUMBER`
    pairs of the keys bam2cns reads are taken, nothing is evaluated."""
    out: Dict[str, float] = {}
    with open(path, encoding="latin-1") as fh:
        for line in fh:
            line = line.split("#", 1)[0]
            for k, v in re.findall(r"""['"]([\w-]+)['"]\s*=>\s*([-+]?\d+(?:\.\d*)?(?:[eE][-+]?\d+)?)""", line):
                if k in _CFG_KEYS:
                    out[k] = float(v)
    return out


def die(msg: str) -> "NoReturn":  # noqa: F821
    print(f"[bam2cns] {msg}", file=sys.stderr)
    sys.exit(255)


@dataclasses.dataclass
class Job:
    """One bam2cns command line: a chunk of long reads and where its output goes."""
    params: cns.CnsParams
    aln_path: str
    aln_fmt: str                      # "bam" | "sam"
    reads: List[cns.LongRead]
    prefix: str
    append: bool
    debug: bool


def prepare(argv: Sequence[str]) -> Job:
    """Parse one bam2cns command line and read its reference chunk (bam2cns:207-322)."""
    a = parse_args(list(argv))
    if not (a.bam or a.sam):
        die("BAM file required")
    for flag, what in ((a.utg_mode, "--utg-mode"), (a.rep_coverage is not None, "--rep-coverage"),
                       (a.min_ncscore is not None, "--min-ncscore"), (a.qual_weighted, "--qual-weighted")):
        if flag:
            die(f"{what} (utg/ccs modes) is not supported by the GPU consensus")
    if a.haplo_coverage:
        die("haploc_consensus??")   # bam2cns:432 dies the same way
    params = cns.CnsParams(
        coverage=cns.parse_perl_number(a.coverage), max_ins_length=a.max_ins_length,
        qv_offset=int(a.qv_offset), use_ref_qual=a.use_ref_qual, detect_chimera=a.detect_chimera,
        invert_scores=a.invert_scores,
    )
    if a.cfg:
        try:
            cfg = read_cfg(a.cfg)
        except OSError as e:
            die(str(e))
        if "sr-trim" in cfg:
            params.trim = int(cfg["sr-trim"])
        if "sr-indel-taboo-length" in cfg:
            params.indel_taboo_length = int(cfg["sr-indel-taboo-length"])
        if "sr-indel-taboo" in cfg:
            params.indel_taboo = cfg["sr-indel-taboo"]
        if "debug" in cfg and not any(x in ("--debug", "--no-debug") for x in argv):
            a.debug = bool(cfg["debug"])
    if a.fallback_phred is not None:
        params.fallback_phred = a.fallback_phred
    aln_path = a.bam or a.sam
    if not os.path.exists(aln_path):
        die(f"{aln_path}: no such file")
    ignore_mcr = a.ignore_mcr
    reads: List[cns.LongRead] = []
    if a.ref:
        hits = sorted(glob.glob(a.ref))
        if not hits:
            die(f"Reference file not found ({a.ref})")
        ref_file = hits[0]
        with open(ref_file, "rb") as fh:
            c0 = fh.read(1)
        if c0 == b"@":
            po = guess_phred_offset(ref_file)
            if po is not None and po != params.qv_offset:
                die(f"Detected [{po}] and specified [{params.qv_offset}] phred offsets differ!")
        elif c0 != b">":
            die(f"Unknown format of reference file: {ref_file}")
        reads, is_fastq = read_refs(ref_file, a.ref_offset, int(a.max_ref_seqs or 0))
        if not is_fastq:
            params.use_ref_qual = False   # bam2cns:258
            ignore_mcr = True             # bam2cns:259-262
    # Without --ref, bam2cns:313-320 fills %LR from the @SQ header but never @LR_IDS,
    # so no read is processed and the output files stay empty: same here.
    if ignore_mcr:
        for r in reads:
            r.desc = ""
    reads.sort(key=functools.cmp_to_key(lambda x, y: byfile_cmp(x.id, y.id)))
    return Job(params, aln_path, "bam" if a.bam else "sam", reads, a.prefix, a.append, a.debug)


def execute(jobs: Sequence[Job]) -> None:
    """Run jobs, batching every job that shares an alignment file and parameters
    into one GPU launch (one pass over the alignment file per batch)."""
    groups: Dict[tuple, List[Job]] = {}
    for j in jobs:
        groups.setdefault((j.aln_path, j.aln_fmt, dataclasses.astuple(j.params)), []).append(j)
    for (path, fmt, _), js in groups.items():
        reads = [r for j in js for r in j.reads]
        if fmt == "bam" and reads and not os.environ.get("PRGPU_BAM2CNS_PYREADER"):
            # one native pass over the BAM (inflate + decode in libprgpu), columns into pr_cns_batch
            try:
                names, cols = bam_alns_native(path)
            except (OSError, ValueError, RuntimeError) as e:
                die(f"{path}: {e}")
            res = cns.run_packed(reads, pack_bam_chunk(reads, names, cols), js[0].params)
            k = 0
            for j in js:
                write_outputs(j, res[k:k + len(j.reads)])
                k += len(j.reads)
            continue
        want: Dict[str, int] = {}
        for i, r in enumerate(reads):
            want.setdefault(r.id, i)
        alns: List[List[cns.SamRecord]] = [[] for _ in reads]
        if reads:
            try:
                _, recs = bam_records(path) if fmt == "bam" else sam_records(path)
                for rec in recs:
                    i = want.get(rec.rname)
                    if i is None:
                        continue
                    if rec.seq == "*":
                        die("Cannot handle BAM secondary alignments without seq/qual")
                    alns[i].append(rec)
            except (OSError, ValueError, struct.error) as e:
                die(f"{path}: {e}")
        # a read id repeated across jobs gets the same alignments (samtools view "id:")
        for i, r in enumerate(reads):
            if want[r.id] != i:
                alns[i] = alns[want[r.id]]
        res = cns.run_chunk(reads, alns, js[0].params) if reads else []
        k = 0
        for j in js:
            write_outputs(j, res[k:k + len(j.reads)])
            k += len(j.reads)


def write_outputs(j: Job, res: Sequence[cns.ReadResult]) -> None:
    """bam2cns:267-285 output files; records as printed at bam2cns:445-455, 488."""
    mode = "a" if j.append else "w"
    pre = j.prefix
    with open(pre + ".fq", mode) as fq, open(pre + ".ignored.tsv", mode), \
            open(pre + ".chim.tsv", mode) as fc:
        tr = open(pre + ".debug.trace", mode) if j.debug else None
        try:
            for r in res:
                if r.status != 0:
                    die(f"{r.id}: consensus failed ({r.status})")
                fq.write(r.fastq)
                if tr:
                    tr.write(r.fastq)
                    tr.write(r.trace + "\n")
                for line in r.chim_lines():
                    fc.write(line + "\n")
        finally:
            if tr:
                tr.close()


def main(argv=None) -> int:
    execute([prepare(sys.argv[1:] if argv is None else argv)])
    return 0


if __name__ == "__main__":
    sys.exit(main())
