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
