"""ctypes binding of the C oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product path never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
LIB = ORACLE_DIR / "liboracle.so"


class OcnsParams(C.Structure):
    _fields_ = [
        ("max_coverage", C.c_double),
        ("bin_size", C.c_double),
        ("trim", C.c_int),
        ("indel_taboo_length", C.c_int),
        ("indel_taboo", C.c_double),
        ("min_aln_length", C.c_int),
        ("max_ins_length", C.c_int),
        ("fallback_phred", C.c_int),
        ("phred_offset", C.c_int),
        ("ref_phred_offset", C.c_int),
        ("use_ref_qual", C.c_int),
        ("qual_weighted", C.c_int),
        ("detect_chimera", C.c_int),
        ("invert_scores", C.c_int),
    ]


class OcnsResult(C.Structure):
    _fields_ = [
        ("fastq", C.c_char_p),
        ("seq", C.c_char_p),
        ("qual", C.c_char_p),
        ("trace", C.c_char_p),
        ("cigar", C.c_char_p),
        ("chim", C.c_char_p),
        ("kept", C.POINTER(C.c_int)),
        ("bin_bases", C.POINTER(C.c_long)),
        ("nbins", C.c_long),
    ]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        _lib.ocns_run.argtypes = [
            C.POINTER(OcnsParams), C.c_char_p, C.c_char_p, C.c_char_p, C.c_long,
            C.POINTER(C.c_char_p), C.c_long, C.POINTER(C.c_long), C.c_int, C.POINTER(OcnsResult)]
        _lib.ocns_run.restype = C.c_int
        _lib.ocns_free.argtypes = [C.POINTER(OcnsResult)]
        _lib.ocns_phred2freq.argtypes = [C.c_int]
        _lib.ocns_phred2freq.restype = C.c_double
        _lib.ocns_freq2phred.argtypes = [C.c_double]
        _lib.ocns_freq2phred.restype = C.c_int
    return _lib


def params_from_case(case, **over):
    p = OcnsParams()
    p.max_coverage = float(case.p("coverage"))
    p.bin_size = 20.0
    p.trim = 1
    p.indel_taboo_length = 7
    p.indel_taboo = 0.1
    p.min_aln_length = 50
    p.max_ins_length = int(case.p("max_ins_length"))
    p.fallback_phred = 1
    p.phred_offset = 33
    p.ref_phred_offset = 33
    p.use_ref_qual = int(case.p("use_ref_qual")) if case.p("noref") != "1" else 0
    p.qual_weighted = int(case.p("qual_weighted"))
    p.detect_chimera = int(case.p("detect_chimera"))
    p.invert_scores = 0
    for k, v in over.items():
        setattr(p, k, v)
    return p


def mcr_ranges(desc):
    import re
    return [(int(a), int(b)) for a, b in re.findall(r"MCR\d+:(\d+),(\d+)", desc)]


def run_case(case):
    """Run the oracle on a casefmt.Case. Returns dict or {'error': rc}."""
    L = lib()
    P = params_from_case(case)
    noref = case.p("noref") == "1"
    seq = case.ref[1]
    qual = case.ref[3]
    ign = [] if noref else mcr_ranges(case.ref_desc)
    flat = (C.c_long * (2 * len(ign) + 1))(*[x for r in ign for x in r])
    lines = (C.c_char_p * (len(case.sam) + 1))(*[s.encode() for s in case.sam])
    R = OcnsResult()
    rc = L.ocns_run(C.byref(P), case.ref_id.encode(), None if noref else seq.encode(),
                    None if noref else qual.encode(), len(seq), lines, len(case.sam),
                    flat, len(ign), C.byref(R))
    out = {"rc": rc}
    if rc == 0:
        out["fastq"] = R.fastq.decode()
        out["trace"] = R.trace.decode()
        out["cigar"] = R.cigar.decode()
        out["chim"] = R.chim.decode()
        out["kept"] = "".join(str(R.kept[i]) for i in range(len(case.sam)))
        out["bin_bases"] = [R.bin_bases[i] for i in range(R.nbins)]
    L.ocns_free(C.byref(R))
    return out


# ---------------------------------------------------------------------------
# SW oracle (oracle/sw_oracle.c)
class OswOpts(C.Structure):
    _fields_ = [("a", C.c_int), ("b", C.c_int), ("o_del", C.c_int), ("o_ins", C.c_int),
                ("e_del", C.c_int), ("e_ins", C.c_int), ("w", C.c_int), ("pen_clip5", C.c_int),
                ("pen_clip3", C.c_int), ("zdrop", C.c_int), ("min_score_per_base", C.c_double)]


class OswResult(C.Structure):
    _fields_ = [("qb", C.c_int), ("qe", C.c_int), ("rb", C.c_int), ("re", C.c_int),
                ("score", C.c_int), ("truesc", C.c_int), ("w", C.c_int), ("global_score", C.c_int),
                ("w2", C.c_int), ("pos", C.c_int), ("n_cigar", C.c_int), ("cigar", C.c_uint32 * 4096),
                ("pass", C.c_int)]


def sw_opts(task="bwa-sr"):
    """proovread.cfg:320-333 (bwa-sr / bwa-sr-finish); zdrop = bwa default 100."""
    o = OswOpts()
    if task == "bwa-sr-finish":
        o.a, o.b, o.o_del, o.o_ins, o.e_del, o.e_ins, o.w = 5, 13, 15, 19, 3, 3, 30
        o.min_score_per_base = 4.0
    else:
        o.a, o.b, o.o_del, o.o_ins, o.e_del, o.e_ins, o.w = 5, 11, 2, 1, 4, 3, 40
        o.min_score_per_base = 2.5
    o.pen_clip5 = o.pen_clip3 = 30
    o.zdrop = 100
    return o


_sw_set = False


def sw_lib():
    global _sw_set
    L = lib()
    if not _sw_set:
        L.osw_task.argtypes = [C.POINTER(OswOpts), C.POINTER(C.c_uint8), C.c_int, C.POINTER(C.c_uint8),
                               C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(OswResult)]
        L.osw_extend.argtypes = [C.c_int, C.POINTER(C.c_uint8), C.c_int, C.POINTER(C.c_uint8), C.c_int,
                                 C.POINTER(C.c_int8), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.c_int] + [C.POINTER(C.c_int)] * 5
        L.osw_global.argtypes = [C.c_int, C.POINTER(C.c_uint8), C.c_int, C.POINTER(C.c_uint8), C.c_int,
                                 C.POINTER(C.c_int8), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.POINTER(C.c_int), C.POINTER(C.c_uint32), C.c_int]
        L.osw_fill_scmat.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_int8)]
        _sw_set = True
    return L


NT4 = {c: i for i, c in enumerate("ACGT")}


def nt4(s):
    return (C.c_uint8 * max(1, len(s)))(*[NT4.get(c, 4) for c in s.upper()])


def sw_task(opts, q, ref, strand, qbeg, rbeg, slen):
    L = sw_lib()
    r = OswResult()
    rc = L.osw_task(C.byref(opts), nt4(q), len(q), nt4(ref), len(ref), strand, qbeg, rbeg, slen, C.byref(r))
    assert rc == 0
    cig = "".join(f"{x >> 4}{'MIDNSHP=X'[x & 15]}" for x in r.cigar[:r.n_cigar])
    return r, cig


def sw_extend(q, t, h0, w=40, a=5, b=11, o_del=2, e_del=4, o_ins=1, e_ins=3, end_bonus=30, zdrop=100):
    L = sw_lib()
    mat = (C.c_int8 * 25)()
    L.osw_fill_scmat(a, b, mat)
    outs = [C.c_int() for _ in range(5)]
    sc = L.osw_extend(len(q), nt4(q), len(t), nt4(t), 5, mat, o_del, e_del, o_ins, e_ins, w, end_bonus,
                      zdrop, h0, *[C.byref(x) for x in outs])
    return sc, [x.value for x in outs]   # qle, tle, gtle, gscore, max_off


# ---------------------------------------------------------------------------
# bwa mem per-read alignment oracle (oracle/aln_oracle.c)
class OswRegion(C.Structure):
    _fields_ = [(k, C.c_int) for k in ("qb", "qe", "rb", "re", "score", "truesc", "w", "seedlen0")]


class OalnSeed(C.Structure):
    _fields_ = [(k, C.c_int) for k in ("sr", "lr", "strand", "qbeg", "rbeg", "slen", "rmax0", "rmax1", "chain",
                                       "rank")]


class OalnOpts(C.Structure):
    _fields_ = [("drop_ratio", C.c_double), ("mask_level", C.c_double), ("mask_level_redun", C.c_double),
                ("max_chain_gap", C.c_int)]


class OalnReg(C.Structure):
    _fields_ = [("lr", C.c_int), ("strand", C.c_int), ("g", OswRegion), ("secondary", C.c_int), ("flag", C.c_int),
                ("seed", C.c_int), ("patched", C.c_int)]


def aln_opts(task="bwa-sr"):
    o = OalnOpts()
    o.drop_ratio = 0.75 if task == "bwa-sr-finish" else 0.0
    o.mask_level, o.mask_level_redun, o.max_chain_gap = 0.5, 0.95, 10000
    return o


_aln_set = False


def aln_lib():
    global _aln_set
    L = sw_lib()
    if not _aln_set:
        L.oaln_read.argtypes = [C.POINTER(OswOpts), C.POINTER(OalnOpts), C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                C.c_int, C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.POINTER(C.c_int),
                                C.POINTER(C.c_int)]
        L.osw_reg2aln.argtypes = [C.POINTER(OswOpts), C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                  C.POINTER(OswRegion), C.POINTER(OswResult)]
        L.osw_extend_seed.argtypes = [C.POINTER(OswOpts), C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                      C.c_int, C.c_int, C.c_int, C.POINTER(OswRegion)]
        _aln_set = True
    return L
