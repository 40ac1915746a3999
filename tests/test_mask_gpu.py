"""Masking on the GPU (mask_lr_kernel through pr_mask_run / pr_iter_mask) against
the oracle's mask_hcrs restatement (oracle/seqfilter_oracle.py, whose HCR search
is pinned to the reference Fastq::Seq::qual_lcs goldens): masked bases, MCR lists
and the (bpt, bpN) statistic, bit-exact.  Host-side parameter parsing and bounds
(no GPU needed) are covered at the end."""
import random
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import seqfilter_oracle as O  # noqa: E402

GOLD = ROOT / "tests" / "golden"


def _cp(P: O.MaskParams):
    from proovread_amd import mask
    p = mask.params()
    p.phred_min, p.phred_max, p.mask_min_len, p.unmask_min_len = P.phred_min, P.phred_max, P.mask_min_len, \
        P.unmask_min_len
    p.mask_reduce, p.end_ratio, p.phred_offset = P.mask_reduce, P.end_ratio, P.phred_offset
    return p


def _seq(rng, L):
    return bytes(rng.choice(b"ACGTacgtN") if rng.random() < 0.02 else rng.choice(b"ACGT") for _ in range(L))


def _check(seqs, quals, P):
    from proovread_amd import mask
    got, mcrs, st = mask.run(seqs, quals, _cp(P))
    want, wmcrs, wst = O.mask_reads(seqs, quals, P)
    assert mcrs == wmcrs
    assert got == want
    assert st == wst
    return sum(len(m) for m in mcrs)


@pytest.mark.gpu
def test_mask_golden_cases():
    rng = random.Random(5)
    by_params = {}
    for line in (GOLD / "seqfilter_cases.txt").read_text().splitlines():
        f = line.split("\t")
        if f[0] == "MASK":
            by_params.setdefault(tuple(f[1:7]), []).append(f[7].encode())
    n = 0
    for key, quals in by_params.items():
        P = O.MaskParams(*map(int, key[:5]), float(key[5]))
        n += _check([_seq(rng, len(q)) for q in quals], quals, P)
    assert n > 50


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_mask_random_batches(seed):
    rng = random.Random(seed)
    for _ in range(6):
        P = O.MaskParams(20, 41, rng.randint(1, 120), rng.randint(0, 200), rng.randint(0, 60),
                         rng.choice([0.0, 0.3, 0.7, 1.0]))
        seqs, quals = [], []
        for _ in range(rng.randint(1, 60)):
            L = rng.choice([0, 1, 63, 64, 65, 500, 2000, 10000])
            q, hi = [], rng.random() < 0.6
            while len(q) < L:
                n = rng.randint(1, rng.choice([20, 300, 3000]))
                q += [rng.randint(53, 74) if hi else rng.randint(33, 52) for _ in range(n)]
                hi = not hi
            quals.append(bytes(q[:L]))
            seqs.append(_seq(rng, L))
        _check(seqs, quals, P)


@pytest.mark.gpu
def test_mask_cfg_default_and_empty():
    from proovread_amd import mask
    assert mask.run([], [], mask.params("20,41,80,130,60,0.7", 150)) == ([], [], (0, 0))
    q = b"J" * 5000
    got, mcrs, st = mask.run([b"A" * 5000], [q], mask.params("20,41,80,130,60,0.7", 150))
    want = O.mask_reads([b"A" * 5000], [q], O.mask_params_from_cfg("20,41,80,130,60,0.7", 150))
    assert (got, mcrs, st) == want
    assert st[1] > 4000


@pytest.mark.gpu
def test_iter_mask_matches_oracle_on_consensus():
    """pr_iter_mask on a resident iteration's consensus vs the oracle on the downloaded
    consensus seq/qual; the device statistic is exactly (bpt, bpN) over status-0 reads."""
    from proovread_amd import _abi, cns, iteration, mask, sw, synth
    d = synth.simulate(77, 60_000, 40, 3000, 50.0, sr_frac=0.3)
    it = iteration.Iteration(d)
    it.launch(sw.default_opts(False), cns.CnsParams(coverage=11.25, use_ref_qual=True))
    p = mask.params("20,41,80,130,60,0.7", 150)
    st = _abi.DevBuffer(it.ctx, 16)
    it.mask_to(st.ptr, p)
    it.sync()
    masked = it.masked()
    a = it.download()
    seqs, quals = [], []
    for i in range(it.n_lr):
        if a["status"][i] == 0:
            o, sl = int(a["out_off"][i]), int(a["seq_len"][i])
            seqs.append(a["seq"][o:o + sl].tobytes())
            quals.append(a["qual"][o:o + sl].tobytes())
    want, _, wst = O.mask_reads(seqs, quals, O.mask_params_from_cfg("20,41,80,130,60,0.7", 150))
    assert [m for m, s in zip(masked, a["status"]) if s == 0] == want
    assert tuple(int(x) for x in st.download(np.int64)) == wst
    assert wst[1] > 0


# ---- host-side ABI (no GPU)

def test_params_parse_matches_proovread_scaling():
    from proovread_amd import mask
    for spec, srl in [("20,41,80,130,60,0.7", 150), ("20,41,80,130,60,0.3", 101), ("20,41,80,130,60,0.7", 100),
                      ("15,40,75,125,30,0.5", 250)]:
        p = mask.params(spec, srl)
        P = O.mask_params_from_cfg(spec, srl)
        assert (p.phred_min, p.phred_max, p.mask_min_len, p.unmask_min_len, p.mask_reduce, p.end_ratio) == \
            (P.phred_min, P.phred_max, P.mask_min_len, P.unmask_min_len, P.mask_reduce, P.end_ratio)
    with pytest.raises(RuntimeError):
        mask.params("20,41,80", 150)


def test_mask_bound_and_validation():
    import ctypes as C
    from proovread_amd import _abi, mask
    L = _abi.lib()
    p = mask.params("20,41,80,130,60,0.7", 150)   # runs >= 240
    off = np.array([0, 0, 239, 240 + 239, 240 + 239 + 5000], np.int64)
    cap = C.c_int64()
    _abi.check(L.pr_mask_bound(C.byref(p), 4, off.ctypes.data, C.byref(cap)), "bound")
    assert cap.value == sum(int(x) // 240 + 2 for x in np.diff(off))
    p.mask_min_len = 0
    assert L.pr_mask_bound(C.byref(p), 4, off.ctypes.data, C.byref(cap)) == -1
