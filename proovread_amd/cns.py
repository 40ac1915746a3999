"""Consensus stage host layer: what one `bam2cns` worker does for a chunk of
long reads (bin/bam2cns:216-455), executed by libprgpu.so on the GPU.

Mirrors the reference interface:

* ``CnsParams`` carries the Sam::Seq class globals that bam2cns sets
  (bam2cns:227-237: Trim, InDelTabooLength, InDelTaboo, MaxCoverage, BinSize,
  MaxInsLength, FallbackPhred) and the consensus() options (use_ref_qual,
  ignore_coords from MCR tags, qual_weighted) plus --detect-chimera.
* ``run_chunk(reads, alignments)`` == one bam2cns invocation: every long read
  of the chunk (natural-sorted ids, bam2cns:324), its alignments in BAM order,
  one GPU launch for all of them.  Results carry the FASTQ record
  (bam2cns:453), the trace / CIGAR (`.debug.trace`, bam2cns:441-444) and the
  chimera lines (`.chim.tsv`, bam2cns:488).
* ``SamSeq`` is a small object with the Sam::Seq method names
  (new / add_aln_by_score / consensus / chimera) for single-read use.

Errors: a read whose alignments would make the Perl engine die returns a
status != 0 (see include/prgpu.h PR_ERR_*); run_chunk raises like bam2cns
exits with 255 (Verbose->exit) unless ``raise_on_error=False``.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import re
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _abi

CIGAR_OPS = {"M": 0, "I": 1, "D": 2, "N": 3, "S": 4, "H": 5, "P": 6, "=": 7, "X": 8}
_CIG_RE = re.compile(r"(\d+)([MIDNSHP=X])")
_NUM_RE = re.compile(r"\s*([+-]?(?:\d+\.?\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?))")


@dataclasses.dataclass
class CnsParams:
    """Sam::Seq class globals + consensus() options (Seq.pm:114-128, bam2cns:171-237)."""
    coverage: float = 50.0            # --coverage -> MaxCoverage
    bin_size: float = 20.0            # BinSize; bam2cns:186 never parses --bin-size
    trim: int = 1                     # cfg sr-trim
    indel_taboo_length: int = 7       # cfg sr-indel-taboo-length
    indel_taboo: float = 0.1          # cfg sr-indel-taboo
    min_aln_length: int = 50          # StateMatrixMinAlnLength
    max_ins_length: int = 0           # --max-ins-length
    fallback_phred: int = 1           # --fallback-phred
    phred_offset: int = 33            # Sam::Seq PhredOffset (consensus output)
    qv_offset: int = 33               # --qv-offset (reference FASTQ)
    use_ref_qual: bool = True         # --[no-]use-ref-qual
    qual_weighted: bool = False       # --qual-weighted
    detect_chimera: bool = False      # --detect-chimera
    invert_scores: bool = False       # --invert-scores

    def to_c(self) -> _abi.CnsParams:
        p = _abi.CnsParams()
        p.max_coverage = float(self.coverage)
        p.bin_size = float(self.bin_size)
        p.trim = int(self.trim)
        p.indel_taboo_length = int(self.indel_taboo_length or 0)
        p.indel_taboo = float(self.indel_taboo)
        p.min_aln_length = int(self.min_aln_length)
        p.max_ins_length = int(self.max_ins_length)
        p.fallback_phred = int(self.fallback_phred)
        p.phred_offset = int(self.phred_offset)
        p.ref_phred_offset = int(self.qv_offset)
        p.use_ref_qual = int(bool(self.use_ref_qual))
        p.qual_weighted = int(bool(self.qual_weighted))
        p.detect_chimera = int(bool(self.detect_chimera))
        p.invert_scores = int(bool(self.invert_scores))
        return p


@dataclasses.dataclass
class LongRead:
    id: str
    seq: Optional[str]          # None: no --ref (lengths from the SAM header)
    qual: Optional[str] = None
    desc: str = ""
    length: Optional[int] = None

    @property
    def len(self) -> int:
        return len(self.seq) if self.seq is not None else int(self.length)

    def mcr_ranges(self) -> List[Tuple[int, int]]:
        """bam2cns:382-391 MCRn:off,len tags of the reference description."""
        return [(int(a), int(b)) for a, b in re.findall(r"MCR\d+:(\d+),(\d+)", self.desc or "")]


@dataclasses.dataclass
class ReadResult:
    id: str
    status: int
    seq: str = ""
    qual: str = ""
    trace: str = ""
    cigar: List[Tuple[int, str]] = dataclasses.field(default_factory=list)
    chim: List[Tuple[int, int, int, int]] = dataclasses.field(default_factory=list)
    kept: Optional[np.ndarray] = None
    bin_bases: Optional[np.ndarray] = None

    @property
    def fastq(self) -> str:
        """Fastq::Seq string (Fastq/Seq.pm:1270-1291) as printed at bam2cns:453."""
        return f"@{self.id}\n{self.seq}\n+\n{self.qual}\n"

    @property
    def cigar_str(self) -> str:
        return "".join(f"{n}{op}" for n, op in self.cigar)

    def chim_lines(self) -> List[str]:
        """bam2cns:488 printf("%s\\t%d\\t%d\\t%s\\n") with Perl number stringification."""
        out = []
        for fr, to, npos, ntot in self.chim:
            out.append(f"{self.id}\t{fr}\t{to}\t{perl_num(npos / ntot)}")
        return out


def perl_num(x: float) -> str:
    """Perl's default stringification of an NV (%.15g)."""
    s = "%.15g" % x
    return s


def parse_perl_number(s: str) -> float:
    m = _NUM_RE.match(s)
    return float(m.group(1)) if m else 0.0


def parse_cigar(cig: str) -> List[int]:
    if cig == "*":
        return []
    ops = []
    pos = 0
    for m in _CIG_RE.finditer(cig):
        if m.start() != pos:
            raise ValueError(f"bad CIGAR {cig!r}")
        ops.append((int(m.group(1)) << 4) | CIGAR_OPS[m.group(2)])
        pos = m.end()
    if pos != len(cig):
        raise ValueError(f"bad CIGAR {cig!r}")
    return ops


@dataclasses.dataclass
class SamRecord:
    """The fields of a SAM line the consensus stage reads (Alignment.pm:87-110)."""
    rname: str
    pos: int
    cigar: List[int]
    seq: str
    qual: str
    score: Optional[float]

    @classmethod
    def from_line(cls, line: str) -> "SamRecord":
        f = line.rstrip("\n").split("\t", 11)
        if len(f) < 11:
            raise ValueError("SAM line with < 11 fields")
        score = None
        if len(f) == 12:
            for t in f[11].split("\t"):
                if t[:2] == "AS":
                    score = parse_perl_number(t[5:])
        return cls(f[2], int(f[3]), parse_cigar(f[5]), f[9], f[10], score)


def pack_chunk(reads: Sequence[LongRead], alns: Sequence[Sequence[SamRecord]]) -> Dict[str, np.ndarray]:
    """Flatten a chunk into the SoA arrays of pr_cns_batch."""
    d = pack_reads(reads)
    d.update(pack_alns(alns))
    return d


def pack_reads(reads: Sequence[LongRead]) -> Dict[str, np.ndarray]:
    """The long-read part of pr_cns_batch: lengths, reference seq / qual, MCR ranges."""
    n = len(reads)
    lens = np.array([r.len for r in reads], dtype=np.int64)
    lr_off = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=lr_off[1:])
    has_ref = n > 0 and all(r.seq is not None for r in reads)
    d: Dict[str, np.ndarray] = {"lr_off": lr_off}
    if has_ref:
        d["ref_seq"] = np.frombuffer("".join(r.seq for r in reads).encode("latin-1"), np.uint8).copy()
        quals = []
        for r in reads:
            q = r.qual or ""
            # a quality string shorter than the sequence contributes nothing past its end
            # (Seq.pm:262 `next unless $freqs[$i]`): pad with phred 0
            quals.append(q[: len(r.seq)] + chr(33) * max(0, len(r.seq) - len(q)))
        d["ref_qual"] = np.frombuffer("".join(quals).encode("latin-1"), np.uint8).copy()
    ign = [r.mcr_ranges() if has_ref else [] for r in reads]
    if any(ign):
        ig_off = np.zeros(n + 1, np.int64)
        np.cumsum([len(x) for x in ign], out=ig_off[1:])
        d["ign_off"] = ig_off
        d["ign"] = np.array([v for x in ign for rg in x for v in rg] or [0], np.int32)
    return d


def pack_alns(alns: Sequence[Sequence[SamRecord]]) -> Dict[str, np.ndarray]:
    """The alignment part of pr_cns_batch: every read's SAM records in BAM order."""
    d: Dict[str, np.ndarray] = {}
    n = len(alns)
    counts = [len(a) for a in alns]
    aln_off = np.zeros(n + 1, np.int64)
    np.cumsum(counts, out=aln_off[1:])
    na = int(aln_off[-1])
    pos = np.zeros(na, np.int32)
    score = np.zeros(na, np.float64)
    flags = np.zeros(na, np.uint8)
    seq_off = np.zeros(na, np.int64)
    lseq = np.zeros(na, np.int32)
    cig_off = np.zeros(na, np.int64)
    ncig = np.zeros(na, np.int32)
    seqs, quals, cigs = [], [], []
    so = co = 0
    k = 0
    for a_list in alns:
        for a in a_list:
            pos[k] = a.pos
            fl = 0
            if a.score is not None:
                fl |= _abi.PR_ALN_HAS_SCORE
                score[k] = a.score
            if a.seq == "*":
                fl |= _abi.PR_ALN_NO_SEQ
                s = ""
            else:
                s = a.seq
            if a.qual == "*":
                fl |= _abi.PR_ALN_NO_QUAL
                q = chr(33) * len(s)
            else:
                q = a.qual[: len(s)] + chr(33) * max(0, len(s) - len(a.qual))
            flags[k] = fl
            seq_off[k] = so
            lseq[k] = len(s)
            seqs.append(s)
            quals.append(q)
            so += len(s)
            cig_off[k] = co
            ncig[k] = len(a.cigar)
            cigs.extend(a.cigar)
            co += len(a.cigar)
            k += 1
    d.update(aln_off=aln_off, aln_pos=pos, aln_score=score, aln_flags=flags, aln_seq_off=seq_off,
             aln_lseq=lseq, aln_cig_off=cig_off, aln_ncig=ncig)
    d["seq_pool"] = np.frombuffer(("".join(seqs) or "\0").encode("latin-1"), np.uint8).copy()
    d["qual_pool"] = np.frombuffer(("".join(quals) or "\0").encode("latin-1"), np.uint8).copy()
    d["cig_pool"] = np.array(cigs or [0], np.uint32)
    d["_seq_pool_len"] = np.array([so], np.int64)
    d["_cig_pool_len"] = np.array([co], np.int64)
    return d


def make_c_batch(d: Dict[str, np.ndarray]) -> _abi.CnsBatch:
    b = _abi.CnsBatch()
    P = _abi.ptr
    b.n_lr = len(d["lr_off"]) - 1
    b.lr_off = P(d["lr_off"], C.c_int64)
    b.ref_seq = P(d.get("ref_seq"), C.c_uint8)
    b.ref_qual = P(d.get("ref_qual"), C.c_uint8)
    b.ign_off = P(d.get("ign_off"), C.c_int64)
    b.ign = P(d.get("ign"), C.c_int32)
    b.aln_off = P(d["aln_off"], C.c_int64)
    b.aln_pos = P(d["aln_pos"], C.c_int32)
    b.aln_score = P(d["aln_score"], C.c_double)
    b.aln_flags = P(d["aln_flags"], C.c_uint8)
    b.aln_seq_off = P(d["aln_seq_off"], C.c_int64)
    b.aln_lseq = P(d["aln_lseq"], C.c_int32)
    b.aln_cig_off = P(d["aln_cig_off"], C.c_int64)
    b.aln_ncig = P(d["aln_ncig"], C.c_int32)
    b.seq_pool = P(d["seq_pool"], C.c_uint8)
    b.qual_pool = P(d["qual_pool"], C.c_uint8)
    b.cig_pool = P(d["cig_pool"], C.c_uint32)
    b.seq_pool_len = int(d["_seq_pool_len"][0]) if "_seq_pool_len" in d else len(d["seq_pool"])
    b.cig_pool_len = int(d["_cig_pool_len"][0]) if "_cig_pool_len" in d else len(d["cig_pool"])
    return b


class OutBuffers:
    """Host output buffers sized by pr_cns_bounds_of."""

    def __init__(self, d: Dict[str, np.ndarray], cb: _abi.CnsBatch, bin_size: float = 20.0):
        L = _abi.lib()
        bd = _abi.CnsBounds()
        _abi.check(L.pr_cns_bounds_of(C.byref(cb), C.byref(bd)), "pr_cns_bounds_of")
        n = cb.n_lr
        na = int(d["aln_off"][-1])
        lens = np.diff(d["lr_off"])
        self.n_bins = (np.floor(lens / bin_size).astype(np.int64) + 1) if n else np.zeros(0, np.int64)
        self.a = dict(
            out_off=np.zeros(n + 1, np.int64), status=np.zeros(n, np.int32), seq_len=np.zeros(n, np.int32),
            trace_len=np.zeros(n, np.int32), ncigar=np.zeros(n, np.int32), nchim=np.zeros(n, np.int32),
            seq=np.zeros(bd.seq_cap + 1, np.uint8), qual=np.zeros(bd.seq_cap + 1, np.uint8),
            trace=np.zeros(bd.seq_cap + 1, np.uint8), cigar=np.zeros(bd.seq_cap + 1, np.uint32),
            chim_off=np.zeros(n + 1, np.int64), chim=np.zeros(4 * (bd.chim_cap + 1), np.int32),
            kept=np.zeros(na + 1, np.uint8), bin_bases=np.zeros(int(self.n_bins.sum()) + 1, np.int64),
        )
        o = _abi.CnsOut()
        P = _abi.ptr
        a = self.a
        o.out_off = P(a["out_off"], C.c_int64)
        o.status = P(a["status"], C.c_int32)
        o.seq_len = P(a["seq_len"], C.c_int32)
        o.trace_len = P(a["trace_len"], C.c_int32)
        o.ncigar = P(a["ncigar"], C.c_int32)
        o.nchim = P(a["nchim"], C.c_int32)
        o.seq = P(a["seq"], C.c_uint8)
        o.qual = P(a["qual"], C.c_uint8)
        o.trace = P(a["trace"], C.c_uint8)
        o.cigar = P(a["cigar"], C.c_uint32)
        o.chim_off = P(a["chim_off"], C.c_int64)
        o.chim = P(a["chim"], C.c_int32)
        o.kept = P(a["kept"], C.c_uint8)
        o.bin_bases = P(a["bin_bases"], C.c_int64)
        self.c = o

    def results(self, ids: Sequence[str], d: Dict[str, np.ndarray]) -> List[ReadResult]:
        a = self.a
        out = []
        boff = np.zeros(len(ids) + 1, np.int64)
        np.cumsum(self.n_bins, out=boff[1:])
        for i, rid in enumerate(ids):
            st = int(a["status"][i])
            r = ReadResult(rid, st)
            a0, a1 = int(d["aln_off"][i]), int(d["aln_off"][i + 1])
            r.kept = a["kept"][a0:a1].copy()
            if st == 0:
                o = int(a["out_off"][i])
                sl, tl, nc = int(a["seq_len"][i]), int(a["trace_len"][i]), int(a["ncigar"][i])
                r.seq = a["seq"][o:o + sl].tobytes().decode("latin-1")
                r.qual = a["qual"][o:o + sl].tobytes().decode("latin-1")
                r.trace = a["trace"][o:o + tl].tobytes().decode("latin-1")
                ops = a["cigar"][o:o + nc]
                r.cigar = [(int(x >> 4), "MID"[int(x & 15)]) for x in ops]
                c0 = int(a["chim_off"][i])
                nch = int(a["nchim"][i])
                ch = a["chim"][4 * c0:4 * (c0 + nch)].reshape(-1, 4)
                r.chim = [tuple(int(v) for v in row) for row in ch]
                r.bin_bases = a["bin_bases"][boff[i]:boff[i + 1]].copy()
            out.append(r)
        return out


def run_chunk(reads: Sequence[LongRead], alns: Sequence[Sequence[SamRecord]], params: CnsParams,
              ctx: Optional[_abi.Context] = None, raise_on_error: bool = False) -> List[ReadResult]:
    """One bam2cns chunk on the GPU (bin/bam2cns:332-365 for every read)."""
    return run_packed(reads, pack_chunk(reads, alns), params, ctx, raise_on_error)


def run_packed(reads: Sequence[LongRead], d: Dict[str, np.ndarray], params: CnsParams,
               ctx: Optional[_abi.Context] = None, raise_on_error: bool = False) -> List[ReadResult]:
    """run_chunk on an already packed batch (pack_reads + the alignment columns)."""
    ctx = ctx or _abi.default_context()
    cb = make_c_batch(d)
    ob = OutBuffers(d, cb, params.bin_size)
    pc = params.to_c()
    _abi.check(_abi.lib().pr_cns_run(ctx.h, C.byref(pc), C.byref(cb), C.byref(ob.c)), "pr_cns_run")
    res = ob.results([r.id for r in reads], d)
    if raise_on_error:
        for r in res:
            if r.status != 0:
                raise RuntimeError(f"{r.id}: {_abi.ERRORS.get(r.status, r.status)}")
    return res


class SamSeq:
    """Sam::Seq-like facade for a single long read (Seq.pm:495 new, 582
    add_aln_by_score, 714 consensus, 774 chimera).  Computation happens on the
    GPU when consensus() is called."""

    def __init__(self, id: str, len: int, ref: Optional[LongRead] = None, params: Optional[CnsParams] = None):
        self.id = id
        self.len = len
        self.ref = ref
        self.params = params or CnsParams()
        self._alns: List[SamRecord] = []
        self._result: Optional[ReadResult] = None

    def add_aln_by_score(self, aln) -> None:
        if isinstance(aln, str):
            aln = SamRecord.from_line(aln)
        self._alns.append(aln)
        self._result = None

    def _run(self, **kw) -> ReadResult:
        p = dataclasses.replace(self.params, **kw)
        lr = self.ref if self.ref is not None else LongRead(self.id, None, None, "", self.len)
        r = run_chunk([lr], [self._alns], p)[0]
        if r.status != 0:
            raise RuntimeError(f"{self.id}: {_abi.ERRORS.get(r.status, r.status)}")
        return r

    def consensus(self, use_ref_qual: bool = False, qual_weighted: bool = False) -> ReadResult:
        self._result = self._run(use_ref_qual=use_ref_qual, qual_weighted=qual_weighted, detect_chimera=False)
        return self._result

    def chimera(self) -> List[Tuple[int, int, int, int]]:
        return self._run(use_ref_qual=False, detect_chimera=True).chim
