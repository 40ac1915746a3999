"""Host seeding front end (proovread_amd/csrc/seed.cpp via the C-ABI) against the
pure-Python oracle (oracle/seed_oracle.py): substring occurrence counts, bwt_smem1a
SMEM sets, and the full per-read task lists (SMEM rounds, occurrence sampling,
chaining, chain filtering, best seed and chain window) for both proovread option
sets (bwa-sr, bwa-sr-finish).  The oracle counts occurrences by plain string
search, independent of the library's 12-mer index.  Parity with bwa-proovread
itself is unpinned (its source is absent)."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import seed_oracle as so  # noqa: E402

from proovread_amd import seed  # noqa: E402


def _mutate(rng, g, p_ins=0.09, p_del=0.045, p_sub=0.015):
    out = []
    for c in g:
        u = rng.random()
        if u < p_del:
            continue
        if u < p_del + p_sub:
            c = (c + rng.integers(1, 4)) % 4
        out.append(int(c))
        while rng.random() < p_ins:
            out.append(int(rng.integers(0, 4)))
    return out


@pytest.fixture(scope="module")
def data():
    rng = np.random.default_rng(7)
    G = rng.integers(0, 4, 5000)
    rep = G[1000:1200].copy()
    lrs = []
    for i in range(6):
        s = int(rng.integers(0, 3500))
        lr = _mutate(rng, G[s:s + 1500])
        if i % 2:
            lr[100:100] = list(rep)     # a repeat shared by several long reads
        if i == 3:
            for j in rng.integers(0, len(lr), 5):
                lr[j] = 4              # N
        lrs.append(lr)
    srs = []
    for i in range(40):
        s = int(rng.integers(0, 4850))
        r = [int(x) for x in G[s:s + 150]]
        if rng.random() < 0.3:
            r[int(rng.integers(0, 150))] = (r[0] + 1) % 4
        if rng.random() < 0.5:
            r = [3 - x for x in reversed(r)]
        srs.append(r)
    srs.append([int(x) for x in rep[:150]])      # a read from the repeat
    lr_off = np.concatenate([[0], np.cumsum([len(x) for x in lrs])]).astype(np.int64)
    sr_off = np.concatenate([[0], np.cumsum([len(x) for x in srs])]).astype(np.int64)
    return dict(lrs=lrs, srs=srs, lr_seq=np.concatenate([np.array(x, np.uint8) for x in lrs]), lr_off=lr_off,
                sr_seq=np.concatenate([np.array(x, np.uint8) for x in srs]), sr_off=sr_off,
                oidx=so.Index(lrs), G=G)


@pytest.fixture(scope="module")
def index(data):
    return seed.SeedIndex(data["lr_seq"], data["lr_off"])


def test_occ_matches_string_search(data, index):
    rng = np.random.default_rng(1)
    I = data["oidx"]
    for _ in range(400):
        n = int(rng.integers(1, 26))
        if rng.random() < 0.7:
            lr = data["lrs"][int(rng.integers(0, 6))]
            a = int(rng.integers(0, len(lr) - n))
            s = [c if c < 4 else 0 for c in lr[a:a + n]]
            if rng.random() < 0.5:
                s = [3 - c for c in reversed(s)]
        else:
            s = [int(c) for c in rng.integers(0, 4, n)]
        want = I.occ("".join("ACGT"[c] for c in s))
        assert index.occ(np.array(s, np.uint8)) == want, s


def test_smem_matches_oracle(data, index):
    rng = np.random.default_rng(2)
    I = data["oidx"]
    for r in data["srs"][:25]:
        q = np.array(r, np.uint8)
        for x in rng.integers(0, len(r), 3):
            for mi in (1, 3):
                got = index.smem(q, int(x), mi)
                want = so.smem1(I, r, int(x), mi)
                assert (got[0], got[1]) == (want[0], want[1]), (x, mi)


def _cmp(data, index, opts, oopts):
    tasks = index.map(data["sr_seq"], data["sr_off"], opts, threads=4)
    got = [tuple(int(t[k]) for k in seed.TASK_DTYPE.names) for t in tasks]
    want = []
    for i, r in enumerate(data["srs"]):
        want += [tuple(t[k] for k in seed.TASK_DTYPE.names) for t in so.map_read(data["oidx"], oopts, r, i)]
    assert got == want
    return tasks


def test_map_matches_oracle_iteration(data, index):
    tasks = _cmp(data, index, seed.default_opts(False), so.Opts())
    assert len(tasks) > 20


def test_map_matches_oracle_finish(data, index):
    _cmp(data, index, seed.default_opts(True), so.Opts.finish())


def test_map_matches_oracle_sampling_and_drop(data, index):
    """max_occ sampling of repeated seeds (-c) and chain dropping (-D)."""
    o = seed.default_opts(False)
    o.max_occ, o.drop_ratio, o.min_chain_weight = 2, 0.5, 12
    oo = so.Opts(max_occ=2, drop_ratio=0.5, min_chain_weight=12)
    _cmp(data, index, o, oo)


def test_seeds_are_exact_matches(data, index):
    tasks = index.map(data["sr_seq"], data["sr_off"], seed.default_opts(False), threads=2)
    for t in tasks:
        r = data["srs"][t["sr"]]
        lr = data["lrs"][t["lr"]]
        ref = lr if t["strand"] == 0 else [3 - c if c < 4 else 4 for c in reversed(lr)]
        q = r[t["qbeg"]:t["qbeg"] + t["slen"]]
        assert q == ref[t["rbeg"]:t["rbeg"] + t["slen"]]
        assert t["slen"] >= 12 and 0 <= t["rmax0"] <= t["rbeg"] and t["rbeg"] + t["slen"] <= t["rmax1"] <= len(lr)


def test_with_seeded_tasks_groups_by_long_read():
    """bench --seeds host|gpu: the front end's tasks replace the simulation truth, grouped by
    long read (the hand-off's layout), a long read's tasks kept in read / chain order."""
    from proovread_amd import seed as seeding, synth
    d = synth.simulate(9, 60_000, 60, 4000, 30.0, sr_frac=0.5)
    ix = seeding.SeedIndex(d.lr_seq, d.lr_off)
    tasks = ix.map(d.sr_seq, d.sr_off)
    d2 = synth.with_seeded_tasks(d, tasks)
    assert len(d2.t_lr) == len(tasks) > 0
    assert np.all(np.diff(d2.t_lr) >= 0)
    for lr in np.unique(d2.t_lr)[:20]:
        sel = tasks[tasks["lr"] == lr]
        m = d2.t_lr == lr
        assert np.array_equal(d2.t_sr[m], sel["sr"]) and np.array_equal(d2.t_rbeg[m], sel["rbeg"])
    assert d2.sr_seq is d.sr_seq and d2.lr_seq is d.lr_seq


# Digests of the index tables (pr_seed_index_digest) recorded with the single-threaded-fill
# build of round 1 (before the parallel text / count / tail passes and the uninitialised
# big tables): every later build must reproduce them exactly.
INDEX_DIGESTS = {"edge": [3546541225710248283, 8536593745191129070, 10635058001152306152, 10887004318922434826, 17265816249920140396, 10474070083008801549], "s3": [5932085080177065250, 12668374040756329347, 3287268347065411532, 15991074188727081827, 10713618094517999836, 13382138088525873941], "s4": [4197478436865662894, 6759494015559495109, 12608834300269571323, 13333961972377079611, 10616757141662657057, 560078664211191469]}


def _edge_shard():
    rng = np.random.default_rng(7)
    reads = [rng.integers(0, 4, n).astype(np.uint8) for n in (0, 5, 11, 12, 13, 40, 1000, 5000)]
    r = rng.integers(0, 4, 3000).astype(np.uint8)
    r[100:130] = 4
    r[2000] = 4
    reads.append(r)
    off = np.zeros(len(reads) + 1, np.int64)
    np.cumsum([len(x) for x in reads], out=off[1:])
    return np.concatenate(reads), off


@pytest.mark.parametrize("name", ["edge", "s3", "s4"])
def test_index_tables_unchanged(name):
    from proovread_amd import seed, synth
    if name == "edge":
        s, o = _edge_shard()
    else:
        sd, gl, n = {"s3": (3, 200_000, 200), "s4": (4, 1_000_000, 1500)}[name]
        d = synth.simulate(sd, gl, n, 5000, 10.0, sr_frac=0.1)
        s, o = d.lr_seq, d.lr_off
    ix = seed.SeedIndex(s, o)
    assert ix.digest() == tuple(INDEX_DIGESTS[name])
    ix.close()
