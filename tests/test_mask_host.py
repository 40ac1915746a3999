"""Masking: the scalar core the GPU kernel runs
(proovread_amd/csrc/mask_core.h), compiled for the host with the wave ballot
emulated (tests/native/mask_host.cpp), against

  * the golden HCR lists of the reference's Fastq::Seq::qual_lcs
    (tests/golden/seqfilter_expected.txt, made by gen_seqfilter_golden.pl), and
  * the oracle's mask_hcrs restatement of sam2cns:806-951 (MCR lists), on the
    golden cases and on random quality strings that drive the iterative gap loop.

Bit-exact offsets and lengths."""
import ctypes as C
import random
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import seqfilter_oracle as O  # noqa: E402

GOLD = ROOT / "tests" / "golden"


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = tmp_path_factory.mktemp("mask") / "libmask_host.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", str(out),
                    str(ROOT / "tests" / "native" / "mask_host.cpp")], check=True)
    L = C.CDLL(str(out))
    L.mask_host.argtypes = [C.c_char_p, C.c_int64] + [C.c_int] * 6 + [C.c_double, C.c_void_p, C.c_void_p,
                                                                       C.c_void_p, C.c_void_p]
    return L


def run(lib, qual: bytes, P: O.MaskParams):
    L = len(qual)
    cap = L // max(P.mask_min_len + 2 * P.mask_reduce, 1) + 2
    f, m = (C.c_int32 * (2 * cap))(), (C.c_int32 * (2 * cap))()
    nf, nm = C.c_int64(), C.c_int64()
    rc = lib.mask_host(qual, L, P.phred_min + 33, P.phred_max + 33, P.mask_min_len + 2 * P.mask_reduce,
                       P.mask_min_len, P.unmask_min_len, P.mask_reduce, P.end_ratio, f, C.byref(nf), m, C.byref(nm))
    assert rc == 0
    pairs = lambda a, n: [[a[2 * i], a[2 * i + 1]] for i in range(n)]
    return pairs(f, nf.value), pairs(m, nm.value)


def golden_cases():
    cases = (GOLD / "seqfilter_cases.txt").read_text().splitlines()
    exp = (GOLD / "seqfilter_expected.txt").read_text().splitlines()
    assert len(cases) == len(exp)
    return [(c.split("\t"), e.split("\t")) for c, e in zip(cases, exp) if c.startswith("MASK")]


def _parse_pairs(s):
    return [[int(x) for x in p.split(",")] for p in s.split()] if s else []


def test_oracle_qual_lcs_matches_reference():
    n = 0
    for f, e in golden_cases():
        pmin, pmax, mm, um, red = map(int, f[1:6])
        got = O.qual_lcs(f[7].encode(), pmin + 33, pmax + 33, mm + 2 * red)
        assert got == _parse_pairs(e[1])
        n += 1
    assert n == 98


def test_core_matches_goldens_and_oracle(lib):
    n_mcr = 0
    for f, e in golden_cases():
        P = O.MaskParams(*map(int, f[1:6]), float(f[6]))
        q = f[7].encode()
        found, mcr = run(lib, q, P)
        assert found == _parse_pairs(e[1])
        assert mcr == O.mask_hcrs(q, P)[1]
        n_mcr += len(mcr)
    assert n_mcr > 50


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_core_matches_oracle_random(lib, seed):
    rng = random.Random(seed)
    rounds = 0
    for _ in range(400):
        P = O.MaskParams(20, 41, rng.randint(1, 60), rng.randint(0, 120), rng.randint(0, 20),
                         rng.choice([0.0, 0.3, 0.5, 0.7, 1.0]))
        L = rng.choice([1, 5, 64, 65, 127, 128, 129, 300, 1000, 3000])
        q, hi = [], rng.random() < 0.5
        while len(q) < L:
            n = rng.randint(1, rng.choice([8, 40, 200]))
            q += [rng.randint(53, 74) if hi else rng.randint(33, 52)] * n
            hi = not hi
        q = bytes(q[:L])
        found, mcr = run(lib, q, P)
        want_found, want = O.mask_hcrs(q, P)
        assert found == O.qual_lcs(q, 53, 74, P.mask_min_len + 2 * P.mask_reduce)
        assert mcr == want, (P, q)
        rounds += len(want_found) > len(want)
    assert rounds > 30   # cases where the gap rounds dropped HCRs


def test_mask_params_from_cfg():
    P = O.mask_params_from_cfg("20,41,80,130,60,0.7", 150)
    assert (P.mask_min_len, P.unmask_min_len, P.mask_reduce, P.end_ratio) == (120, 195, 60, 0.7)
    P = O.mask_params_from_cfg("20,41,80,130,60,0.3", 101)
    assert (P.mask_min_len, P.unmask_min_len) == (81, 131)
