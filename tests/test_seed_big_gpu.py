"""Seed index beyond 2^32 text positions (configs[3]: 270 k x 10 kb = 2.7 Gb of long reads, a
5.4 G-position text with both strands; SURVEY.md §8d C4, §8e exact-parity layout: every rank
holds the index of ALL long reads).

Positions are stored as their low 32 bits; a k-mer's hits beyond 2^32 form the tail of its
list from ksplit[code] on (seed_core.h).  The device build sorts the text in 2^30-position
chunks behind a global histogram (seed_index.hip).

The long-read set: reads A (genomic), 2.2 G bases of N padding, reads B (genomic).  The text is
forward reads, then the reverse complement of their concatenation, so A's reverse strand lies
beyond 2^32 and B's forward strand near 2^31: short reads from A's loci seed at positions on
both sides of 2^32.  Checked: the device seeds (pr_seed_gpu_index_build + pr_seed_gpu_map)
equal the host path's (pr_seed_index_build + pr_seed_map, seed_core.h on the CPU) seed for
seed, and seeds on A's reverse strand exist.  A second test sends a small text through the
chunked device build (PRGPU_INDEX_CHUNK) and checks its tables' digests against the host
build's.  (bwa mode's seeding order depends on global occurrence counts, so equality with the
host path over the whole index is the bar, not equality with a smaller index.)"""
import os

import numpy as np
import pytest

PAD = 2_200_000_000


def big_long_reads():
    from proovread_amd import synth
    d = synth.simulate(20261017, 300_000, 60, 5000, 20, sr_frac=0.05)
    n = d.n_lr
    a = [d.lr_seq[d.lr_off[i]:d.lr_off[i + 1]] for i in range(0, n, 2)]
    b = [d.lr_seq[d.lr_off[i]:d.lr_off[i + 1]] for i in range(1, n, 2)]
    npad = 22
    lens = [len(x) for x in a] + [PAD // npad] * npad + [len(x) for x in b]
    off = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    seq = np.full(int(off[-1]), 4, np.uint8)
    k = 0
    for x in a:
        seq[off[k]:off[k + 1]] = x
        k += 1
    k += npad
    for x in b:
        seq[off[k]:off[k + 1]] = x
        k += 1
    return d, seq, off, len(a), npad


def host_tasks(seq, off, sr, sr_off, finish=False):
    from proovread_amd import seed
    ix = seed.SeedIndex(seq, off)
    try:
        return ix.map(sr, sr_off, seed.default_opts(finish), threads=16)
    finally:
        ix.close()


def test_host_index_beyond_2_32_equals_unpadded():
    """CPU: N padding adds no k-mer and keeps the text order of everything else, so the paged
    host index gives the seeds of the same reads without the padding (long-read ids shifted)."""
    d, seq, off, na, npad = big_long_reads()
    want = host_tasks(seq, off, d.sr_seq, d.sr_off)
    keep = np.r_[0:na, na + npad:len(off) - 1]
    parts = [seq[off[i]:off[i + 1]] for i in keep]
    o2 = np.zeros(len(parts) + 1, np.int64)
    np.cumsum([len(x) for x in parts], out=o2[1:])
    ref = host_tasks(np.concatenate(parts), o2, d.sr_seq, d.sr_off)
    got = want.copy()
    got["lr"][got["lr"] >= na] -= npad
    for f in got.dtype.names:
        assert np.array_equal(got[f], ref[f]), f
    assert ((want["lr"] < na) & (want["strand"] == 1)).sum() > 100


@pytest.mark.gpu
@pytest.mark.parametrize("finish", [False, True])
def test_device_index_beyond_2_32_matches_host(finish):
    from proovread_amd import _abi, seed
    d, seq, off, na, npad = big_long_reads()
    n_text = 2 * int(off[-1]) + 2 * (len(off) - 1)
    assert n_text > 2 ** 32
    sr, sr_off = d.sr_seq, d.sr_off
    want = host_tasks(seq, off, sr, sr_off, finish)
    hx = seed.SeedIndex(seq, off)
    want_digest = hx.digest()
    hx.close()
    # a context of its own, destroyed at the end: a >2^32-position index holds
    # ~100 GB that later tests in the same process need back
    ctx = _abi.Context(int(os.environ.get("LOCAL_RANK", "-1")))
    try:
        ix = seed.DeviceSeedIndex(ctx, seq, off)
        assert ix.digest() == want_digest   # every table, ksplit included
        got, st = ix.map(sr, sr_off, seed.default_opts(finish))
    finally:
        ctx.close()
    assert (st == 0).all()
    assert len(want) > d.n_sr
    for f in ("sr", "lr", "strand", "qbeg", "rbeg", "slen", "rmax0", "rmax1", "chain", "rank"):
        assert np.array_equal(got[f], want[f]), f
    # seeds on A's reverse strand: text positions beyond 2^32
    assert ((want["lr"] < na) & (want["strand"] == 1)).sum() > 100
    assert ((want["lr"] >= na + npad) & (want["strand"] == 0)).sum() > 100


@pytest.mark.gpu
def test_chunked_device_build_matches_host_tables(monkeypatch):
    from proovread_amd import _abi, seed, synth
    d = synth.simulate(23, 2_000_000, 300, 6000, 1.0, sr_frac=0.01)
    hx = seed.SeedIndex(d.lr_seq, d.lr_off)
    want = hx.digest()
    hx.close()
    monkeypatch.setenv("PRGPU_INDEX_CHUNK", "20")   # 2^20-position sorts: 4 chunks
    ctx = _abi.default_context()
    ix = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
    assert ix.digest() == want
