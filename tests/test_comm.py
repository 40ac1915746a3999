"""The product's collectives (comm.RcclComm over libprgpu's pr_comm_*, RCCL on the library's
own HIP runtime) and their file rendezvous.

The reference has no collective; the multi-GPU loop's only data-path one is
the all-reduce of the per-iteration {bpt, bpN} statistic (mask_shortcut_frac's input,
bin/proovread:1702-1720, 2026-2047), plus the exact-parity layout's all-gather / all-to-all.
CPU: the rendezvous (key, atomic publish, wait, timeout).  GPU: a world-1 communicator built
through the same rendezvous, every collective against numpy, and the iteration's device
statistic all-reduced in place (one GPU per box: world > 1 is covered by the gloo tests of
the same loop, test_correct_loop.py / test_cns_shard.py / test_exact_shard.py)."""
import os
import threading
import time

import numpy as np
import pytest

from proovread_amd import comm


def test_rendezvous_key_names_job_and_attempt(monkeypatch, tmp_path):
    monkeypatch.delenv("PRGPU_RDZV_KEY", raising=False)
    monkeypatch.setenv("PRGPU_RDZV_DIR", str(tmp_path))
    monkeypatch.setenv("MASTER_PORT", "29501")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job7")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    p0 = comm.rendezvous_path()
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    p1 = comm.rendezvous_path()
    assert p0 != p1 and p0.parent == tmp_path
    assert str(os.getppid()) in p0.name and "29501" in p0.name and "job7" in p0.name
    monkeypatch.setenv("PRGPU_RDZV_KEY", "explicit")
    assert comm.rendezvous_path().name == "prgpu_rdzv_explicit.id"


def test_exchange_id_publishes_atomically(monkeypatch, tmp_path):
    monkeypatch.setenv("PRGPU_RDZV_DIR", str(tmp_path))
    idb = bytes(range(comm.ID_BYTES))
    got = {}

    def reader(r):
        got[r] = comm.exchange_id(r, None, key="t1", timeout=20)

    ths = [threading.Thread(target=reader, args=(r,)) for r in (1, 2, 3)]
    for t in ths:
        t.start()
    time.sleep(0.1)
    assert comm.exchange_id(0, lambda: idb, key="t1") == idb
    for t in ths:
        t.join()
    assert got == {1: idb, 2: idb, 3: idb}
    assert not list(tmp_path.glob("*.tmp*"))   # the temporary file was renamed, never left


def test_wait_for_ignores_partial_and_times_out(tmp_path):
    p = tmp_path / "x.id"
    p.write_bytes(b"short")
    with pytest.raises(TimeoutError):
        comm.wait_for(p, comm.ID_BYTES, timeout=0.2)


def test_pack_unpack_lists_roundtrip():
    items = [b"", b"a", bytes(300), b"xyz"]
    assert comm._unpack_lists([comm._pack_list(items), comm._pack_list([]), comm._pack_list([b"q"])]) == items + [b"q"]


@pytest.mark.gpu
def test_rccl_world1_collectives(monkeypatch, tmp_path):
    from proovread_amd import _abi
    monkeypatch.setenv("PRGPU_RDZV_DIR", str(tmp_path))
    ctx = _abi.default_context()
    cm = comm.RcclComm(ctx, 0, 1, key="w1")
    try:
        assert not list(tmp_path.glob("prgpu_rdzv_*"))   # rank 0 removed the id once all ranks had it
        cm.barrier()
        # device buffer, in place on the context stream: {bpt, bpN} and the other dtypes / ops
        v = np.array([123456789012, 98765], np.int64)
        buf = _abi.DevBuffer(ctx, 16)
        buf.upload(v)
        for op in (comm.RED_SUM, comm.RED_MAX, comm.RED_MIN):
            cm.allreduce_dev(buf.ptr, 2, comm.DT_I64, op)
        assert np.array_equal(buf.download(np.int64), v)
        f = np.array([1.5, -2.25, 3e300, 0.0], np.float64)
        fb = _abi.DevBuffer(ctx, f.nbytes)
        fb.upload(f)
        cm.allreduce_dev(fb.ptr, len(f), comm.DT_F64, comm.RED_SUM)
        assert np.array_equal(fb.download(np.float64), f)
        cm.allreduce_dev(fb.ptr, 0, comm.DT_F64, comm.RED_SUM)   # zero elements
        # host buffers
        assert cm.allreduce_ints([7, -3, 1 << 40]) == [7, -3, 1 << 40]
        assert cm.allreduce_ints([5], comm.RED_MAX) == [5]
        assert cm.allreduce_floats([0.25, 1e-300], comm.RED_MIN) == [0.25, 1e-300]
        # variable-size all-gather, including empty blocks
        assert cm.allgather_bytes(b"") == [b""]
        assert cm.allgather_bytes(bytes(range(256)) * 5) == [bytes(range(256)) * 5]
        assert cm.allgather_lists([b"", b"ab", bytes(1000)]) == [b"", b"ab", bytes(1000)]
        # all-to-all: the self send/recv pair of ncclSend/ncclRecv, and a zero-length block
        rows = np.arange(60, dtype=np.int32).reshape(20, 3)
        assert np.array_equal(cm.alltoallv_rows(rows, np.array([20])), rows)
        assert cm.alltoallv_rows(np.zeros((0, 3), np.int32), np.array([0])).shape == (0, 3)
        # a staging buffer grown after a small call (re-allocation on the context's device)
        big = np.arange(1 << 18, dtype=np.int64)
        assert cm.allreduce_ints(big.tolist()[:70000]) == big.tolist()[:70000]
    finally:
        cm.close()


@pytest.mark.gpu
def test_rccl_allreduce_of_iteration_statistic(monkeypatch, tmp_path):
    """The bench / loop step's statistic: pr_iter_mask fills {bpt, bpN} on the device, the
    world-1 all-reduce leaves it unchanged, and it equals the masked reads' own counts."""
    from proovread_amd import _abi, cns, iteration, mask, sw, synth
    monkeypatch.setenv("PRGPU_RDZV_DIR", str(tmp_path))
    ctx = _abi.default_context()
    d = synth.simulate(77, 30000, 12, 2500, 15, sr_frac=1.0)
    it = iteration.Iteration(d, ctx=ctx)
    it.launch(sw.default_opts(False), cns.CnsParams(coverage=11.25, use_ref_qual=True))
    stats = _abi.DevBuffer(ctx, 16)
    it.mask_to(stats.ptr, mask.params("20,41,80,130,60,0.7", 150))
    cm = comm.RcclComm(ctx, 0, 1, key="w1s")
    try:
        cm.allreduce_dev(stats.ptr, 2)
        it.sync()
        bpt, bpn = (int(x) for x in stats.download(np.int64))
    finally:
        cm.close()
    masked = it.masked()
    assert bpt == sum(len(m) for m in masked) > 0
    assert bpn == sum(m.count(b"N") for m in masked)
