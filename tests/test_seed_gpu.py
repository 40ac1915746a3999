"""GPU seeding path (seed_kernels.hip: seed_core.h, one lane per read, fixed scratch).

CPU: the same core with the device's fixed capacities, run on the host
(pr_seed_map_device_caps), gives exactly the host path's tasks for every read it
does not flag, and flags only reads whose work outgrows a capacity.
GPU: pr_seed_gpu_map returns exactly the host run of the device path: tasks and
per-read flags (run last: not yet exercised on hardware)."""
import numpy as np
import pytest

from proovread_amd import seed, synth


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
