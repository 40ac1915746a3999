"""The exact-parity multi-GPU layout on the device (include/prgpu.h pr_aln_exchange; SURVEY.md
§8e): short-read shards aligned against ALL long reads, every reported alignment packed on the
device and sent to the owner of its long read (RCCL all-to-all of device buffers, or device
copies between the contexts of one process), then -b/-l filter + hand-off + consensus on the
owner.  No SAM text, no per-alignment host code.

Bar: byte-for-byte the single-GPU iteration (pr_iter_*, which the CPU chain pins in
test_iter_gpu.py) on every owned long read -- corrected sequence, qualities, trace, consensus
CIGAR, chimera records, masked reads and the {bpt, bpN} statistic:

  * world 1 without a communicator and with an RCCL one (self send/recv through RCCL);
  * worlds 2, 3 and 5 of contexts on one GPU (pr_aln_exchange_local: the same packs and
    regrouping, device copies in place of RCCL -- one GPU per box here, so RCCL at world > 1
    runs only on the driver's 8-GPU node).

The reference's layout is one bwa-proovread over all reads, then bam2cns per chunk
(bin/proovread:1313, 1596-1619); the shards are contiguous and the blocks arrive
source-rank-major, so the owner sees every long read's alignments in the single run's order."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ASCII = np.frombuffer(b"ACGTN", np.uint8)


def _data(finish):
    from proovread_amd import synth
    # finish: reads as after the iterations (the finish scoring rejects raw 15 % CLR alignments)
    err = dict(p_ins=0.02, p_del=0.01, p_sub=0.005) if finish else {}
    d = synth.simulate(71 + finish, 60000, 48, 3000, 30, sr_frac=1.0, **err)
    ref = ASCII[d.lr_seq]
    rng = np.random.default_rng(5)
    qual = (rng.integers(0, 30, len(ref)) + 33).astype(np.uint8)
    return d, ref, qual


def _opts(finish):
    from proovread_amd import cns, seed, sw
    so = sw.default_opts(finish=finish)
    so.bin_size, so.bin_length = 20, 20.0 * (30 if finish else 15)
    cp = cns.CnsParams(coverage=22.5 if finish else 11.25, use_ref_qual=not finish, detect_chimera=finish)
    return seed.default_opts(finish), so, cp


def _outputs(it, mask_params):
    from proovread_amd import _abi
    res = it.results()
    buf = _abi.DevBuffer(it.ctx, 16)
    it.mask_to(buf.ptr, mask_params)
    masked = it.masked()
    st = buf.download(np.int64)
    buf.close()
    return [(r.status, r.seq, r.qual, r.trace, r.cigar, r.chim) for r in res], masked, [int(x) for x in st[:2]]


def _single(ctx, d, ref, qual, finish, mask_params):
    from proovread_amd import iteration, seed
    seed_opts, so, cp = _opts(finish)
    ix = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
    ix.map(d.sr_seq, d.sr_off, seed_opts, keep_on_device=True)
    it = iteration.Iteration(d, lr_qual=qual, ctx=ctx, ref_seq=ref, gpu_seeds=True)
    it.launch(so, cp)
    return _outputs(it, mask_params)


def _shard(ctx, d, finish, s, e, device_pools=False):
    from proovread_amd import iteration, seed
    seed_opts, so, _ = _opts(finish)
    ix = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
    a, b = int(d.sr_off[s]), int(d.sr_off[e])
    ix.map(d.sr_seq[a:b], d.sr_off[s:e + 1] - a, seed_opts, keep_on_device=True)
    iteration.ShardSW(ctx, d.sr_seq, d.sr_off, s, e, d.lr_seq, d.lr_off, device_pools=device_pools).launch(so)


def _owned(ctx, d, ref, qual, finish, lo, hi, mask_params, sr=True):
    from proovread_amd import iteration
    _, so, cp = _opts(finish)
    it = iteration.OwnedIteration(ctx, lo, hi, d.lr_off, ref, qual, d.sr_seq if sr else None, d.sr_off)
    it.launch(so, cp)
    return _outputs(it, mask_params)


def _mask_params():
    from proovread_amd import mask
    return mask.params("20,41,80,130,60,0.7", 150)


@pytest.mark.parametrize("finish", [False, True])
@pytest.mark.parametrize("transport", ["none", "rccl"])
def test_world1_exchange_equals_single_iteration(finish, transport, monkeypatch, tmp_path):
    """The whole exchange (pack, counts, RCCL self send/recv -- or a device copy --, regroup) at
    world 1, forced (without PRGPU_XCHG_FORCE world 1 passes the SW output straight through)."""
    from proovread_amd import _abi, comm, iteration
    ctx = _abi.default_context()
    d, ref, qual = _data(finish)
    mp = _mask_params()
    want = _single(ctx, d, ref, qual, finish, mp)
    assert sum(1 for x in want[0] if x[0] == 0) == d.n_lr
    monkeypatch.setenv("PRGPU_XCHG_FORCE", "1")   # world 1 would skip the identity exchange
    cm = None
    if transport == "rccl":
        monkeypatch.setenv("PRGPU_RDZV_DIR", str(tmp_path))
        cm = comm.RcclComm(ctx, 0, 1, key=f"xchg{int(finish)}")
    try:
        _shard(ctx, d, finish, 0, d.n_sr)
        bounds = np.array([0, d.n_lr], np.int64)
        n = iteration.exchange(ctx, cm, 0, bounds)
        assert n > 10 * d.n_lr
        got = _owned(ctx, d, ref, qual, finish, 0, d.n_lr, mp)
    finally:
        if cm is not None:
            cm.close()
    assert got[0] == want[0]
    assert got[1] == want[1]
    assert got[2] == want[2]


@pytest.mark.parametrize("world", [2, 3, 5])
@pytest.mark.parametrize("finish", [False, True])
def test_local_exchange_equals_single_iteration(world, finish):
    """`world` shards as contexts of this process on one GPU: the owners' results concatenated
    in rank order equal the single iteration's; the {bpt, bpN} sums too.  Even worlds take the
    SW pools and the consensus reference from the device (the seeding's copies, the SW's long
    reads); the single run uses the ASCII reference of the same bases."""
    from proovread_amd import _abi, exact_shard as ex, iteration
    d, ref, qual = _data(finish)
    mp = _mask_params()
    ctx0 = _abi.default_context()
    want = _single(ctx0, d, ref, qual, finish, mp)
    ctxs = [_abi.Context(0) for _ in range(world)]
    try:
        bounds = ex.lr_bounds(d.lr_off, world)
        starts = []
        for r in range(world):
            s, e = ex.sr_range(d.n_sr, world, r)
            _shard(ctxs[r], d, finish, s, e, device_pools=world % 2 == 0)
            starts.append(s)
        nrecv = iteration.exchange_local(ctxs, starts, bounds)
        assert sum(nrecv) > 10 * d.n_lr
        res, masked, st = [], [], [0, 0]
        for r in range(world):
            g = _owned(ctxs[r], d, None if world % 2 == 0 else ref, qual, finish, int(bounds[r]), int(bounds[r + 1]),
                       mp)
            res += g[0]
            masked += g[1]
            st = [st[0] + g[2][0], st[1] + g[2][1]]
    finally:
        for c in ctxs:
            c.close()
    assert len(res) == d.n_lr
    assert res == want[0]
    assert masked == want[1]
    assert st == want[2]


@pytest.mark.parametrize("finish", [False, True])
def test_world1_passthrough_equals_single_iteration(finish):
    """World 1 without the test hook: the owned launch takes the SW output directly."""
    from proovread_amd import _abi, iteration
    ctx = _abi.default_context()
    d, ref, qual = _data(finish)
    mp = _mask_params()
    want = _single(ctx, d, ref, qual, finish, mp)
    _shard(ctx, d, finish, 0, d.n_sr, device_pools=True)
    iteration.exchange(ctx, None, 0, np.array([0, d.n_lr], np.int64))
    got = _owned(ctx, d, None, qual, finish, 0, d.n_lr, mp, sr=False)   # every pool from the device
    assert got == want
