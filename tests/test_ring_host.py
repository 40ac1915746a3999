"""The register-ring ksw_extend2 of the GPU extension kernel
(proovread_amd/csrc/sw_ring.h), compiled for the host as one lane, against the
C oracle's ksw_extend2 restatement (oracle/sw_oracle.c osw_extend) on random
query/target pairs: every band class the kernel instantiates (WB 32/40/64/80),
both bwa-proovread scoring sets, z-drop on/off, h0 and end-bonus variants.
Bit-exact: score, qle, tle, gtle, gscore, max_off."""
import ctypes as C
import random
import subprocess
from pathlib import Path

import pytest

import oracle_bind as ob

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def ring(tmp_path_factory):
    out = tmp_path_factory.mktemp("ring") / "libring_host.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", str(out),
                    str(ROOT / "tests" / "native" / "ring_host.cpp")], check=True)
    return C.CDLL(str(out))


def _nt4(s):
    return (C.c_uint8 * max(1, len(s)))(*[{"A": 0, "C": 1, "G": 2, "T": 3}.get(c, 4) for c in s])


def _mutate(s, rng, p):
    o = []
    for c in s:
        r = rng.random()
        if r < p * 0.3:
            continue
        if r < p * 0.6:
            o += [rng.choice("ACGT"), c]
        elif r < p:
            o.append(rng.choice("ACGTN"))
        else:
            o.append(c)
    return "".join(o)


SCORING = [(5, 11, 2, 4, 1, 3, 100), (5, 13, 15, 3, 19, 3, 100), (1, 4, 6, 1, 6, 1, 0)]
BANDS = {10: 32, 25: 32, 32: 32, 40: 40, 60: 64, 80: 80}


@pytest.mark.parametrize("seed", [11, 12])
def test_ring_matches_oracle(ring, seed):
    rng = random.Random(seed)
    n = 0
    for _ in range(500):
        L = rng.choice([1, 2, 5, 10, 20, 40, 60, 75, 100, 150, 200])
        q = "".join(rng.choice("ACGT") for _ in range(L))
        t = _mutate(q, rng, rng.choice([0, 0.05, 0.15, 0.3])) + \
            "".join(rng.choice("ACGT") for _ in range(rng.randint(0, 60)))
        if rng.random() < 0.2:
            t = "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 200)))
        w = rng.choice(list(BANDS))
        h0 = rng.choice([0, 5, 30, 100, 400])
        eb = rng.choice([30, 0, 5])
        for a, b, od, ed, oi, ei, zd in SCORING:
            sc, outs = ob.sw_extend(q, t, h0, w=w, a=a, b=b, o_del=od, e_del=ed, o_ins=oi, e_ins=ei,
                                    end_bonus=eb, zdrop=zd)
            o5 = (C.c_int * 5)()
            sc2 = ring.ring_extend(BANDS[w], a, b, od, ed, oi, ei, zd, len(q), _nt4(q), len(t), _nt4(t),
                                   w, eb, h0, o5)
            assert (sc2, list(o5)) == (sc, outs), (q, t, w, h0, eb, (a, b, od, ed, oi, ei, zd))
            n += 1
    assert n == 1500


@pytest.mark.parametrize("seed", [21, 22])
def test_global_ring_matches_oracle(ring, seed):
    """ksw_global2 + backtrack on the register ring vs oracle osw_global: score and CIGAR."""
    L = ob.sw_lib()
    rng = random.Random(seed)
    n = 0
    for _ in range(400):
        lq = rng.choice([1, 2, 5, 10, 30, 60, 100, 150, 200])
        q = "".join(rng.choice("ACGT") for _ in range(lq))
        t = _mutate(q, rng, rng.choice([0, 0.05, 0.15, 0.3])) or "A"
        dl = abs(len(t) - len(q))
        wb = rng.choice([40, 80])
        if dl + 3 > wb:
            continue
        w = rng.randint(dl + 3, wb)
        for a, b, od, ed, oi, ei, _ in SCORING[:2]:
            mat = (C.c_int8 * 25)()
            L.osw_fill_scmat(a, b, mat)
            nc, cig = C.c_int(), (C.c_uint32 * 4096)()
            sc = L.osw_global(len(q), _nt4(q), len(t), _nt4(t), 5, mat, od, ed, oi, ei, w, C.byref(nc), cig, 4096)
            nc2, cig2 = C.c_int(), (C.c_uint32 * 4096)()
            sc2 = ring.ring_global(wb, a, b, od, ed, oi, ei, len(q), _nt4(q), len(t), _nt4(t), w,
                                   C.byref(nc2), cig2, 4096)
            assert (sc2, list(cig2[:nc2.value])) == (sc, list(cig[:nc.value])), (q, t, w, wb)
            n += 1
    assert n > 600
