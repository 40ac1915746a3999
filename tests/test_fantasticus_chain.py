"""configs[0] on the CPU: one bwa-sr correction iteration over the reference's bundled
sample (sample/F.antasticus_long_error.fq: 121 long reads, ~1 kb, PacBio-like errors,
IUPAC codes; fixtures in tests/golden/fantasticus/) with 15x short reads simulated
from sample/F.antasticus_genome.fa (the sample's short-read file is not in the
checkout).  The product's host seeding front end (pr_seed_map) produces the task
list, the CPU oracle chain (SW oracle -> SAM order -> consensus oracle) corrects.

Checked: every genomic long read is corrected to >= 90 % genome-exact 20-mers
(raw reads: ~5 %), the contamination read is not, and the seeding is deterministic."""
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import cpu_chain  # noqa: E402

from proovread_amd import bwa_proovread as bp  # noqa: E402
from proovread_amd import seed, sw  # noqa: E402

FX = ROOT / "tests" / "golden" / "fantasticus"


def simulate_sr(G, cov, seed_=20261015, L=150):
    rng = np.random.default_rng(seed_)
    n = int(cov * len(G) / L)
    st = rng.integers(0, len(G) - L, n)
    srs = G[st[:, None] + np.arange(L)[None, :]].copy()
    m = rng.random(n) < 0.15
    k = int(m.sum())
    pos = rng.integers(0, L, k)
    srs[np.nonzero(m)[0], pos] = (srs[np.nonzero(m)[0], pos] + 1) % 4
    rev = rng.random(n) < 0.5
    srs[rev] = (3 - srs[rev])[:, ::-1]
    return srs.reshape(-1).astype(np.uint8), np.arange(n + 1, dtype=np.int64) * L


@pytest.fixture(scope="module")
def sample():
    names, seqs, _ = bp.read_fastx(str(FX / "F.antasticus_long_error.fq"))
    _, gs, _ = bp.read_fastx(str(FX / "F.antasticus_genome.fa"))
    G = sw.NT4[np.frombuffer(gs[0], np.uint8)]
    lr_seq, lr_off = bp._pool(seqs)
    sr_seq, sr_off = simulate_sr(G, 15)
    return dict(names=names, seqs=seqs, G=G, lr_seq=lr_seq, lr_off=lr_off, sr_seq=sr_seq, sr_off=sr_off)


def _kmers(G, k=20):
    s = "".join("ACGT"[c] for c in G)
    rc = s[::-1].translate(str.maketrans("ACGT", "TGCA"))
    return {t[i:i + k] for t in (s, rc) for i in range(len(t) - k + 1)}


def _frac(s, km, k=20):
    s = s.upper()
    n = len(s) - k + 1
    return sum(s[i:i + k] in km for i in range(n)) / max(n, 1)


def test_fantasticus_iteration(sample):
    ix = seed.SeedIndex(sample["lr_seq"], sample["lr_off"])
    tk = ix.map(sample["sr_seq"], sample["sr_off"], seed.default_opts(False), threads=4)
    tk2 = ix.map(sample["sr_seq"], sample["sr_off"], seed.default_opts(False), threads=1)
    assert np.array_equal(tk, tk2)
    # bwa mode: every seed of the kept chains, bwa mem's per-read alignment on the oracle
    d = SimpleNamespace(lr_seq=sample["lr_seq"], lr_off=sample["lr_off"], sr_seq=sample["sr_seq"],
                        sr_off=sample["sr_off"], t_sr=tk["sr"].astype(np.int32), t_lr=tk["lr"].astype(np.int32),
                        t_strand=tk["strand"].astype(np.uint8), t_qbeg=tk["qbeg"].astype(np.int32),
                        t_rbeg=tk["rbeg"].astype(np.int32), t_slen=tk["slen"].astype(np.int32),
                        t_chain=tk["chain"].astype(np.int32), n_lr=len(sample["seqs"]),
                        n_sr=len(sample["sr_off"]) - 1)
    _, _, res, _ = cpu_chain.run_sample(d, range(d.n_lr), workers=4)
    km = _kmers(sample["G"])
    for name, raw, (rc, fq) in zip(sample["names"], sample["seqs"], res):
        assert rc == 0
        cor = fq.split("\n")[1]
        fr = _frac(raw.decode(), km)
        fc = _frac(cor, km)
        if name.startswith("long_contamination"):
            assert fc < 0.5, name
        else:
            assert fr < 0.3 and fc >= 0.9, (name, fr, fc)
