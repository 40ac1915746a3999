"""GPU seeding path (seed_kernels.hip: one wave per read, wave-parallel occurrence table,
seed_core.h's SMEM / chaining / filter on lane 0, fixed scratch per wave).

CPU: the same core with the device's fixed capacities, run on the host
(pr_seed_map_device_caps), gives exactly the host path's tasks for every read it
does not flag, and flags only reads whose work outgrows a capacity.
GPU: pr_seed_gpu_map against the pure-Python oracle (oracle/seed_oracle.py: string
search occurrence counts, bwt_smem1a, mem_chain, mem_chain_flt) directly, for both
option sets, -c sampling and -D dropping; and against the host run of the device path
on a larger simulated sample (tasks and per-read flags)."""
import sys
from pathlib import Path

import numpy as np
import pytest

from proovread_amd import seed, synth

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import seed_oracle as so  # noqa: E402


def _data(scale_seed=11, gl=300_000, n_lr=300):
    d = synth.simulate(scale_seed, gl, n_lr, 5000, 40.0, sr_frac=0.3)
    n = min(6000, d.n_sr)
    return d, d.sr_seq[:d.sr_off[n]], d.sr_off[:n + 1]


def _by_read(tasks, n):
    out = [[] for _ in range(n)]
    for t in tasks:
        out[int(t["sr"])].append(tuple(int(x) for x in t))
    return out


@pytest.mark.parametrize("finish", [False, True])
def test_device_caps_core_matches_host_path(finish):
    d, ss, so = _data()
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    o = seed.default_opts(finish)
    host = ix.map(ss, so, o)
    dev, st = ix.map_device_caps(ss, so, o, threads=4)
    n = len(so) - 1
    hb, db = _by_read(host, n), _by_read(dev, n)
    ok = st == 0
    assert ok.mean() > 0.99
    assert all(hb[i] == db[i] for i in range(n) if ok[i])
    assert all(db[i] == [] for i in range(n) if not ok[i])
    assert len(host) > 2 * n


def test_device_caps_core_reads_no_stale_scratch(monkeypatch):
    """Device scratch is never cleared between reads: the core's result must not depend on what
    the slab held before (PRGPU_SCRATCH_FILL poisons the host emulation's slabs)."""
    d, ss, so = _data(12)
    ss, so = ss[:so[2000]], so[:2001]
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    for finish in (False, True):
        o = seed.default_opts(finish)
        want, wst = ix.map_device_caps(ss, so, o, threads=4)
        for fill in ("0xFF", "0xA5"):
            monkeypatch.setenv("PRGPU_SCRATCH_FILL", fill)
            got, st = ix.map_device_caps(ss, so, o, threads=4)
            monkeypatch.delenv("PRGPU_SCRATCH_FILL")
            assert np.array_equal(st, wst) and np.array_equal(got, want), fill


def test_device_caps_flags_long_reads():
    d, _, _ = _data()
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    rng = np.random.default_rng(3)
    L = int(d.lr_off[1] - d.lr_off[0])
    long_read = d.lr_seq[d.lr_off[0]:d.lr_off[0] + min(L, 1500)].astype(np.uint8)   # > 1024: flagged
    short = rng.integers(0, 4, 150).astype(np.uint8)
    ss = np.concatenate([short, long_read])
    so = np.array([0, 150, 150 + len(long_read)], np.int64)
    _, st = ix.map_device_caps(ss, so)
    assert st[0] == 0 and st[1] & 1


@pytest.mark.gpu
def test_gpu_seeding_matches_device_caps_on_host():
    from proovread_amd import _abi
    d, ss, so = _data(12)
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    ctx = _abi.default_context()
    ix.to_gpu(ctx)
    for finish in (False, True):
        o = seed.default_opts(finish)
        want, wst = ix.map_device_caps(ss, so, o)
        got, st = ix.map_gpu(ss, so, o, allow_flagged=True)
        assert np.array_equal(st, wst)
        assert np.array_equal(got, want)
    assert ix.gpu_ms() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("sr_len", [600, 950])
def test_gpu_seeding_mr_reads_match_host_path(sr_len):
    """The mr modes' long short reads (bwa-mr-1 options): mem_flt_chained_seeds' local SW runs
    for every seed of every kept chain (>= 440 bp); the capacities follow the read length and
    the one-wave-per-read pass scores the seeds over all lanes.  Every read is seeded (none
    flagged) and the seeds equal the host path's."""
    from proovread_amd import _abi, tasks as T
    d = synth.simulate(20261017 + sr_len, 300_000, 900, 10_000, 15.0, sr_len=sr_len, sr_frac=1.0)
    n = min(2500, d.n_sr)
    ss, so = d.sr_seq[:d.sr_off[n]], d.sr_off[:n + 1]
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    ix.to_gpu(_abi.default_context())
    o = T.options("bwa-mr-1")[0]
    want = ix.map(ss, so, o, threads=8)
    got, st = ix.map_gpu(ss, so, o, allow_flagged=True)
    assert not st.any()
    assert np.array_equal(got, want)
    assert len(want) > 100 * n


@pytest.mark.gpu
def test_gpu_seeding_in_output_chunks(monkeypatch):
    """Reads mapped in chunks of bounded output slabs (PRGPU_SEED_OUT_MB; 1 MB = 64 reads per
    chunk here, 94 chunks) give the one-chunk run's seeds and flags exactly, kept on the device
    (seed count) and downloaded."""
    from proovread_amd import _abi
    d, ss, so = _data(12)
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    ctx = _abi.default_context()
    ix.to_gpu(ctx)
    o = seed.default_opts(False)
    want, wst = ix.map_gpu(ss, so, o, allow_flagged=True)
    monkeypatch.setenv("PRGPU_SEED_OUT_MB", "1")
    got, st = ix.map_gpu(ss, so, o, allow_flagged=True)
    assert np.array_equal(st, wst)
    assert np.array_equal(got, want)
    if not wst.any():
        seed._map_gpu(ix.L, ctx, ss, so, o, False, keep_on_device=True)
        assert seed._count(ix.L, ctx) == len(want)


@pytest.mark.gpu
def test_gpu_seeding_costliest_first_order(monkeypatch):
    """Pass 1 over the reads sorted costliest first (the opt-in PRGPU_SEED_LPT=1 order): the
    same seeds and flags as read order."""
    from proovread_amd import _abi
    d, ss, so_ = _data(12)
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    ix.to_gpu(_abi.default_context())
    for finish in (False, True):
        o = seed.default_opts(finish)
        monkeypatch.setenv("PRGPU_SEED_LPT", "0")
        want, wst = ix.map_gpu(ss, so_, o, allow_flagged=True)
        monkeypatch.setenv("PRGPU_SEED_LPT", "1")
        got, st = ix.map_gpu(ss, so_, o, allow_flagged=True)
        assert np.array_equal(st, wst) and np.array_equal(got, want)
        assert len(want) > 2 * (len(so_) - 1)


def _oracle_data():
    """Six 1.5 kb long reads with indels, a repeat shared by three of them and N bases;
    41 short reads (substitutions, reverse strands, one from the repeat)."""
    rng = np.random.default_rng(7)
    G = rng.integers(0, 4, 5000)
    rep = G[1000:1200].copy()

    def mutate(g):
        out = []
        for c in g:
            u = rng.random()
            if u < 0.045:
                continue
            if u < 0.06:
                c = (c + rng.integers(1, 4)) % 4
            out.append(int(c))
            while rng.random() < 0.09:
                out.append(int(rng.integers(0, 4)))
        return out
    lrs = []
    for i in range(6):
        s0 = int(rng.integers(0, 3500))
        lr = mutate(G[s0:s0 + 1500])
        if i % 2:
            lr[100:100] = list(rep)
        if i == 3:
            for j in rng.integers(0, len(lr), 5):
                lr[j] = 4
        lrs.append(lr)
    srs = []
    for i in range(40):
        s0 = int(rng.integers(0, 4850))
        r = [int(x) for x in G[s0:s0 + 150]]
        if rng.random() < 0.3:
            r[int(rng.integers(0, 150))] = (r[0] + 1) % 4
        if rng.random() < 0.5:
            r = [3 - x for x in reversed(r)]
        srs.append(r)
    srs.append([int(x) for x in rep[:150]])
    lr_off = np.concatenate([[0], np.cumsum([len(x) for x in lrs])]).astype(np.int64)
    sr_off = np.concatenate([[0], np.cumsum([len(x) for x in srs])]).astype(np.int64)
    return (lrs, srs, np.concatenate([np.array(x, np.uint8) for x in lrs]), lr_off,
            np.concatenate([np.array(x, np.uint8) for x in srs]), sr_off)


@pytest.mark.gpu
def test_gpu_seeding_matches_python_oracle():
    from proovread_amd import _abi
    lrs, srs, lr_seq, lr_off, sr_seq, sr_off = _oracle_data()
    oidx = so.Index(lrs)
    ix = seed.SeedIndex(lr_seq, lr_off)
    ix.to_gpu(_abi.default_context())
    o_samp = seed.default_opts(False)
    o_samp.max_occ, o_samp.drop_ratio, o_samp.min_chain_weight = 2, 0.5, 12
    cases = [(seed.default_opts(False), so.Opts()), (seed.default_opts(True), so.Opts.finish()),
             (o_samp, so.Opts(max_occ=2, drop_ratio=0.5, min_chain_weight=12))]
    for o, oo in cases:
        got, st = ix.map_gpu(sr_seq, sr_off, o)
        assert (st == 0).all()
        got = [tuple(int(t[k]) for k in seed.TASK_DTYPE.names) for t in got]
        want = []
        for i, r in enumerate(srs):
            want += [tuple(t[k] for k in seed.TASK_DTYPE.names) for t in so.map_read(oidx, oo, r, i)]
        assert got == want
        assert len(got) > 20


def _index_cases():
    d, ss, so_ = _data(13, gl=200_000, n_lr=200)
    yield "sim", d.lr_seq, d.lr_off, ss, so_
    lrs, srs, lr_seq, lr_off, sr_seq, sr_off = _oracle_data()
    yield "repeat+N", lr_seq, lr_off, sr_seq, sr_off
    # an empty long read, IUPAC-like codes > 4, a long read shorter than a 12-mer
    rng = np.random.default_rng(5)
    parts = [rng.integers(0, 4, 3000), np.zeros(0, np.int64), rng.integers(0, 6, 800), rng.integers(0, 4, 7),
             rng.integers(0, 4, 2500)]
    seq = np.concatenate(parts).astype(np.uint8)
    off = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
    reads = [seq[100:250], seq[3100:3250], seq[3900:4050][::-1].copy()]
    sro = np.concatenate([[0], np.cumsum([len(x) for x in reads])]).astype(np.int64)
    yield "edge", seq, off, np.concatenate(reads).astype(np.uint8), sro


@pytest.mark.gpu
def test_device_index_build_equals_host_index():
    """pr_seed_gpu_index_build: the host build's tables byte for byte (digests of text, koff,
    kpos, kext, j-mer counts, contig tables), and seeding against it = the host path."""
    from proovread_amd import _abi
    ctx = _abi.default_context()
    for name, lr_seq, lr_off, sr_seq, sr_off in _index_cases():
        hx = seed.SeedIndex(lr_seq, lr_off)
        dx = seed.DeviceSeedIndex(ctx, lr_seq, lr_off)
        assert dx.digest() == hx.digest(), name
        assert dx.build_ms() > 0
        for finish in (False, True):
            o = seed.default_opts(finish)
            want = hx.map(sr_seq, sr_off, o, threads=4)
            got, st = dx.map(sr_seq, sr_off, o)
            assert (st == 0).all(), name
            assert np.array_equal(got, want), name
        hx.close()


@pytest.mark.gpu
def test_gpu_seeding_near_exact_matches_host_path():
    """The finish task's setting (short reads against near-exact long reads at 30x: every 12-mer
    hits ~30 copies, matches run to the read's end, every read outgrows pass 1's hit slices):
    the occurrence table's 64-base text walks and the SMEM / -y count jumps (seed_core.h
    Occ::scan_ge) give the host path's seeds, for both option sets."""
    from proovread_amd import _abi
    d = synth.simulate(17, 150_000, 900, 5000, 40.0, p_ins=0.002, p_del=0.002, p_sub=0.002, sr_frac=0.1)
    n = min(4000, d.n_sr)
    ss, so_ = d.sr_seq[:d.sr_off[n]], d.sr_off[:n + 1]
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    ix.to_gpu(_abi.default_context())
    for finish in (False, True):
        o = seed.default_opts(finish)
        want = ix.map(ss, so_, o, threads=8)
        got, st = ix.map_gpu(ss, so_, o, allow_flagged=False)
        assert (st == 0).all()
        assert np.array_equal(got, want)
        assert len(want) > 10 * n
    ix.close()
