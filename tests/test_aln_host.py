"""bwa mode's per-read logic as the device runs it (proovread_amd/csrc/aln_core.h: the
mem_chain2aln walk with speculative first seeds and resumed rounds, mem_sort_dedup_patch,
mem_mark_primary_se, mem_reg2sam's filters), compiled for the host with the SW oracle's
extensions (tests/native/aln_host.cpp), against the plain restatement oracle/aln_oracle.c:
the same reported regions, in the same SAM order, from the same seeds, with the same FLAG.
bwa-proovread is absent, so parity with it is unpinned; this pins the device logic to the
restatement."""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as ob

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    out = tmp_path_factory.mktemp("aln") / "libaln_host.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off", "-o", str(out),
                    str(ROOT / "tests" / "native" / "aln_host.cpp"), "-x", "c", str(ROOT / "oracle" / "sw_oracle.c")],
                   check=True)
    L = C.CDLL(str(out))
    L.aln_host_run.argtypes = [C.POINTER(ob.OswOpts), C.c_double, C.c_double, C.c_double, C.c_int, C.c_int] + \
        [C.c_void_p] * 2 + [C.c_int] + [C.c_void_p] * 2 + [C.c_int64] + [C.c_void_p] * 7 + [C.c_int64] + \
        [C.c_void_p] * 10
    return L


def _data(seed_, err, finish, n_lr=30, lr_len=2500, cov=15):
    from proovread_amd import seed, synth
    f = err / 0.15
    d = synth.simulate(seed_, 30000, n_lr, lr_len, cov, p_ins=0.09 * f, p_del=0.045 * f, p_sub=0.015 * f)
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    d = synth.with_seeds(d, ix.map(d.sr_seq, d.sr_off, seed.default_opts(finish), threads=4))
    ix.close()
    return d


def _run_host(L, d, task):
    o = ob.sw_opts(task)
    ao = ob.aln_opts(task)
    n = len(d.t_sr)
    P = lambda a: np.ascontiguousarray(a).ctypes.data
    arrs = {k: np.ascontiguousarray(getattr(d, k)) for k in ("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen",
                                                              "t_chain")}
    nout = np.zeros(d.n_sr, np.int32)
    outs = {k: np.zeros(n + 1, np.int32) for k in ("olist", "oflag", "qb", "qe", "rb", "re", "score", "truesc")}
    stats = np.zeros(3, np.int64)
    rc = L.aln_host_run(C.byref(o), ao.drop_ratio, ao.mask_level, ao.mask_level_redun, ao.max_chain_gap, d.n_sr,
                        P(d.sr_off), P(d.sr_seq), d.n_lr, P(d.lr_off), P(d.lr_seq), n,
                        *[P(arrs[k]) for k in ("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen", "t_chain")],
                        0, P(nout), *[P(outs[k]) for k in ("olist", "oflag", "qb", "qe", "rb", "re", "score",
                                                            "truesc")], P(stats))
    assert rc == 0
    first = np.searchsorted(d.t_sr, np.arange(d.n_sr + 1))
    got = []
    for r in range(d.n_sr):
        v = []
        for i in range(int(nout[r])):
            t = int(outs["olist"][first[r] + i])
            v.append((int(d.t_lr[t]), int(d.t_strand[t]), int(outs["oflag"][first[r] + i]), int(outs["qb"][t]),
                      int(outs["qe"][t]), int(outs["rb"][t]), int(outs["re"][t]), int(outs["score"][t]),
                      int(outs["truesc"][t]), t))
        got.append(v)
    return got, stats


@pytest.mark.parametrize("finish,err", [(False, 0.15), (False, 0.05), (True, 0.05), (True, 0.02)])
def test_device_logic_on_host_matches_oracle(host, finish, err):
    import cpu_chain
    d = _data(11 + int(finish) + int(100 * err), err, finish)
    task = "bwa-sr-finish" if finish else "bwa-sr"
    got, stats = _run_host(host, d, task)
    want = cpu_chain.bwa_alignments(d, task)
    for r in range(d.n_sr):
        w = [(a[0], a[1], a[5], a[6], a[7], a[8], a[9], a[4], a[10], a[11]) for a in want[r]]
        assert got[r] == w, r
    assert sum(map(len, got)) > 2 * d.n_lr
    n_chain = len(np.unique(d.t_sr.astype(np.int64) * 65536 + d.t_chain))
    assert stats[0] >= 1 and stats[1] >= n_chain


def test_device_logic_patches_on_host_match_oracle(host):
    """N windows in the long reads split short reads' alignments into colinear regions that
    mem_sort_dedup_patch merges through mem_patch_reg (aln_patch_score in extra rounds)."""
    import cpu_chain
    from proovread_amd import seed, synth
    f = 0.05 / 0.15
    d = synth.simulate(97, 30000, 30, 2500, 15, p_ins=0.09 * f, p_del=0.045 * f, p_sub=0.015 * f)
    rng = np.random.default_rng(5)
    lr = d.lr_seq.copy()
    for i in range(len(d.lr_off) - 1):   # a 10-110 bp N window every ~300 bp
        a, b = int(d.lr_off[i]), int(d.lr_off[i + 1])
        for x in range(a + 100, b - 200, 300):
            x += int(rng.integers(0, 100))
            lr[x:x + int(rng.integers(10, 111))] = 4
    d.lr_seq = lr
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    d = synth.with_seeds(d, ix.map(d.sr_seq, d.sr_off, seed.default_opts(False), threads=4))
    ix.close()
    got, stats = _run_host(host, d, "bwa-sr")
    want = cpu_chain.bwa_alignments(d, "bwa-sr")
    for r in range(d.n_sr):
        w = [(a[0], a[1], a[5], a[6], a[7], a[8], a[9], a[4], a[10], a[11]) for a in want[r]]
        assert got[r] == w, r
    assert stats[2] > 0
