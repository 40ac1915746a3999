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


def _oracle_opts(o: "seed.SeedOpts") -> "so.Opts":
    return so.Opts(min_seed_len=o.min_seed_len, min_chain_weight=o.min_chain_weight, w=o.w,
                   split_factor=o.split_factor, split_width=o.split_width, max_mem_intv=o.max_mem_intv,
                   max_occ=o.max_occ, drop_ratio=o.drop_ratio, max_chain_gap=o.max_chain_gap,
                   mask_level=o.mask_level, a=o.a, o_del=o.o_del, e_del=o.e_del, o_ins=o.o_ins, e_ins=o.e_ins,
                   b=o.b)


def test_flt_threshold_follows_bwa_float_arithmetic():
    """mem_flt_chained_seeds runs from 1.1f * W <= 0.05f * len: 440 bp at -W 20, 880 at -W 40
    (proovread.cfg:343-365: bwa-mr-1 / bwa-mr -W 20, bwa-mr-finish -W 40), never for sr reads."""
    o = so.Opts(min_chain_weight=20)
    assert so.flt_min_score(o, 439) is None and so.flt_min_score(o, 440) == 110
    assert so.flt_min_score(o, 150) is None
    o40 = so.Opts(min_chain_weight=40)
    assert so.flt_min_score(o40, 879) is None and so.flt_min_score(o40, 880) == 220
    assert so.flt_min_score(so.Opts(min_chain_weight=18), 396) == 99


def test_local_sw_known_answers():
    o = so.Opts()
    assert so.local_sw(o, [0, 1, 2, 3], [0, 1, 2, 3]) == 20
    assert so.local_sw(o, [0, 1, 2, 3] * 5, [3, 3]) == 5
    # one deletion inside 20 matches: 20*5 - (o_del + e_del) = 94 > the 10-base side alone (50)
    q = [0, 1, 2, 3, 1] * 4
    t = q[:10] + [2] + q[10:]
    assert so.local_sw(o, q, t) == 100 - 6
    # one insertion: o_ins + e_ins = 4
    assert so.local_sw(o, t, q) == 100 - 4
    assert so.local_sw(o, [4] * 10, [4] * 10) == 0


@pytest.fixture(scope="module")
def mr_data():
    """mr mode (short reads > 150 bp, bin/proovread:637-641): 450-1000 bp reads from a genome
    whose long reads carry CLR errors, a repeat, and pairs of 13-mers of the genome pasted at
    random places (a chain of weight 26 >= -W whose seeds' +-50 bp windows are otherwise
    random: their seed SW scores fall below mem_flt_chained_seeds' minimum of 110)."""
    rng = np.random.default_rng(11)
    G = rng.integers(0, 4, 8000)
    rep = G[2000:2300].copy()
    lrs = []
    for i in range(8):
        s = int(rng.integers(0, 5500))
        lr = _mutate(rng, G[s:s + 2500], 0.12, 0.06, 0.03)
        if i % 3 == 1:
            lr[300:300] = list(rep)
        for _ in range(6):   # two 13-mers 40 bp apart on the genome, random bases between
            a = int(rng.integers(0, 7900))
            at = int(rng.integers(0, len(lr)))
            lr[at:at] = [int(x) for x in G[a:a + 13]] + [int(x) for x in rng.integers(0, 4, 27)] + \
                [int(x) for x in G[a + 40:a + 53]]
        lrs.append(lr)
    srs = []
    for L in (450, 520, 600, 700, 800, 879, 880, 950, 1000, 640):
        s = int(rng.integers(0, 8000 - L))
        r = [int(x) for x in G[s:s + L]]
        for j in rng.integers(0, L, 3):
            r[int(j)] = (r[int(j)] + 1) % 4
        if rng.random() < 0.5:
            r = [3 - x for x in reversed(r)]
        srs.append(r)
    lr_off = np.concatenate([[0], np.cumsum([len(x) for x in lrs])]).astype(np.int64)
    sr_off = np.concatenate([[0], np.cumsum([len(x) for x in srs])]).astype(np.int64)
    return dict(lrs=lrs, srs=srs, lr_seq=np.concatenate([np.array(x, np.uint8) for x in lrs]), lr_off=lr_off,
                sr_seq=np.concatenate([np.array(x, np.uint8) for x in srs]), sr_off=sr_off, oidx=so.Index(lrs))


@pytest.mark.parametrize("task", ["bwa-mr-1", "bwa-mr-finish"])
def test_map_mr_reads_matches_oracle_with_seed_filter(mr_data, task, monkeypatch):
    """mem_flt_chained_seeds on 450-1000 bp reads (bwa-mr-1 / bwa-mr: -W 20, so every read;
    bwa-mr-finish: -W 40, reads >= 880 bp): the host path equals the oracle task for task
    (dropped seeds, srt order by seed SW score, chain windows over the kept seeds), and the
    filter changes the task lists."""
    from proovread_amd import tasks
    o, _ = tasks.options(task)
    ix = seed.SeedIndex(mr_data["lr_seq"], mr_data["lr_off"])
    got = [tuple(int(t[k]) for k in seed.TASK_DTYPE.names)
           for t in ix.map(mr_data["sr_seq"], mr_data["sr_off"], o, threads=4)]
    ix.close()
    oo = _oracle_opts(o)
    want = []
    for i, r in enumerate(mr_data["srs"]):
        want += [tuple(t[k] for k in seed.TASK_DTYPE.names) for t in so.map_read(mr_data["oidx"], oo, r, i)]
    assert got == want and len(got) > 20
    if task == "bwa-mr-1":   # the filter bites: without it, more seeds in another order
        monkeypatch.setattr(so, "flt_min_score", lambda O, n: None)
        plain = []
        for i, r in enumerate(mr_data["srs"]):
            plain += [tuple(t[k] for k in seed.TASK_DTYPE.names) for t in so.map_read(mr_data["oidx"], oo, r, i)]
        assert len(plain) > len(want)


@pytest.fixture(scope="module")
def near_exact():
    """The finish task's setting: short reads against near-exact long reads at ~30x coverage
    (every 12-mer of a read hits ~30 copies, matches run to the read's end), so the SMEM forward
    extension and bwt_seed_strategy1 (-y) count lengths beyond the per-start count table."""
    rng = np.random.default_rng(11)
    G = rng.integers(0, 4, 2400)
    lrs = []
    for i in range(34):
        s = int(rng.integers(0, 900))
        lr = _mutate(rng, G[s:s + 1500], p_ins=0.002, p_del=0.002, p_sub=0.002)
        if i == 5:
            lr[40] = 4   # an N inside a copy
        lrs.append(lr)
    srs = []
    for i in range(24):
        s = int(rng.integers(0, 2250))
        r = [int(x) for x in G[s:s + 150]]
        if i % 5 == 1:
            r[int(rng.integers(0, 150))] = 4   # a read N
        if rng.random() < 0.5:
            r = [3 - x if x < 4 else 4 for x in reversed(r)]
        srs.append(r)
    lr_off = np.concatenate([[0], np.cumsum([len(x) for x in lrs])]).astype(np.int64)
    sr_off = np.concatenate([[0], np.cumsum([len(x) for x in srs])]).astype(np.int64)
    return dict(lrs=lrs, srs=srs, lr_seq=np.concatenate([np.array(x, np.uint8) for x in lrs]), lr_off=lr_off,
                sr_seq=np.concatenate([np.array(x, np.uint8) for x in srs]), sr_off=sr_off,
                oidx=so.Index(lrs), G=G)


@pytest.mark.parametrize("finish", [False, True])
def test_map_near_exact_matches_oracle(near_exact, finish):
    ix = seed.SeedIndex(near_exact["lr_seq"], near_exact["lr_off"])
    try:
        tasks = _cmp(near_exact, ix, seed.default_opts(finish), so.Opts.finish() if finish else so.Opts())
    finally:
        ix.close()
    assert len(tasks) > 100


def test_smem_near_exact_matches_oracle(near_exact):
    ix = seed.SeedIndex(near_exact["lr_seq"], near_exact["lr_off"])
    try:
        for r in near_exact["srs"][:10]:
            q = np.array(r, np.uint8)
            for x in (0, 37, 75):
                for mi in (1, 20, 31):
                    got = ix.smem(q, x, mi)
                    want = so.smem1(near_exact["oidx"], r, x, mi)
                    assert (got[0], got[1]) == (want[0], want[1]), (x, mi)
    finally:
        ix.close()


@pytest.mark.parametrize("finish", [False, True])
def test_device_caps_near_exact_equals_host(near_exact, finish):
    """The device path's core on the host (finish options: the lazy occurrence table, a start's
    hits on first use) gives the host path's seeds on near-exact reads, whatever the scratch held."""
    import os
    ix = seed.SeedIndex(near_exact["lr_seq"], near_exact["lr_off"])
    try:
        o = seed.default_opts(finish)
        want = ix.map(near_exact["sr_seq"], near_exact["sr_off"], o, threads=2)
        for fill in (None, "0xA5"):
            if fill:
                os.environ["PRGPU_SCRATCH_FILL"] = fill
            try:
                got, st = ix.map_device_caps(near_exact["sr_seq"], near_exact["sr_off"], o, threads=2)
            finally:
                os.environ.pop("PRGPU_SCRATCH_FILL", None)
            assert (st == 0).all() and np.array_equal(got, want), fill
    finally:
        ix.close()
