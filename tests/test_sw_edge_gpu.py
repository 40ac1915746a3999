"""Edge cases of the seed-extension stage on the GPU against the SW oracle:
ragged short-read lengths in one batch (36 .. 1000 bp: the packed kernels' per-length
buckets, the 255 bp packed-frame limit, the 32-bit ring / LDS kernels beyond it, the
general CIGAR kernel's HBM row past ~500 bp, up to proovread's 1000 bp short-read limit,
bin/proovread:457; longer reads fail loudly), N bases in short and long reads, CIGARs
longer than their slots (the overflow pass), and an empty task list.  Same bar as
test_sw_gpu.py: bit-exact qb/qe/rb/re, AS, truesc, POS, CIGAR and the -T pass flag."""
import dataclasses

import numpy as np
import pytest

import oracle_bind as ob
from sw_util import gpu_tuple, oracle_results

LENGTHS = (36, 76, 100, 151, 250, 255, 256, 300, 400, 509, 600, 800, 1000)


def merge(parts):
    """One batch from several synth.Datasets (long / short read ids shifted)."""
    lr_seq = np.concatenate([p.lr_seq for p in parts])
    sr_seq = np.concatenate([p.sr_seq for p in parts])
    lr_off, sr_off = [np.zeros(1, np.int64)], [np.zeros(1, np.int64)]
    t = {k: [] for k in ("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen")}
    nl = ns = 0
    for p in parts:
        lr_off.append(p.lr_off[1:] + lr_off[-1][-1])
        sr_off.append(p.sr_off[1:] + sr_off[-1][-1])
        t["t_sr"].append(p.t_sr + ns)
        t["t_lr"].append(p.t_lr + nl)
        for k in ("t_strand", "t_qbeg", "t_rbeg", "t_slen"):
            t[k].append(getattr(p, k))
        nl += p.n_lr
        ns += p.n_sr
    return dataclasses.replace(parts[0], lr_seq=lr_seq, sr_seq=sr_seq, lr_off=np.concatenate(lr_off),
                               sr_off=np.concatenate(sr_off), **{k: np.concatenate(v) for k, v in t.items()})


def ragged(seed=40):
    from proovread_amd import synth
    parts = [synth.simulate(seed + i, 40000, 8, 4000, 6.0 if L < 300 else (3.0 if L < 600 else 2.0), sr_len=L)
             for i, L in enumerate(LENGTHS)]
    d = merge(parts)
    rng = np.random.default_rng(seed)
    d.sr_seq = d.sr_seq.copy()
    d.sr_seq[rng.random(len(d.sr_seq)) < 0.002] = 4
    d.lr_seq = d.lr_seq.copy()
    d.lr_seq[rng.random(len(d.lr_seq)) < 0.001] = 4
    return d


def test_ragged_batch_shape():
    """CPU: the merged batch really mixes every length and keeps seeds inside their reads."""
    d = ragged()
    lq = np.diff(d.sr_off)
    assert set(LENGTHS) <= set(lq[d.t_sr].tolist())
    assert (d.t_qbeg + d.t_slen <= lq[d.t_sr]).all()
    assert (d.t_rbeg + d.t_slen <= np.diff(d.lr_off)[d.t_lr]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("task", ["bwa-sr", "bwa-sr-finish"])
def test_sw_gpu_ragged_lengths_and_ns(task):
    from proovread_amd import sw
    d = ragged()
    res = sw.run(d.sw_input(), sw.default_opts(finish=task.endswith("finish")))
    assert (res["status"] == 0).all()
    lq = np.diff(d.sr_off)[d.t_sr]
    rng = np.random.default_rng(1)
    idx = np.unique(np.concatenate([rng.choice(np.nonzero(lq == L)[0], size=min(150, int((lq == L).sum())),
                                               replace=False) for L in LENGTHS]))
    want = oracle_results(d, ob.sw_opts(task), idx)
    bad = [(int(t), int(lq[t]), w, gpu_tuple(res, t)) for t, w in zip(idx, want) if tuple(w) != gpu_tuple(res, t)]
    assert not bad, bad[:3]


@pytest.mark.gpu
def test_sw_gpu_empty_task_list():
    from proovread_amd import sw, synth
    d = synth.simulate(3, 20000, 4, 2000, 5.0)
    e = dataclasses.replace(d, **{k: getattr(d, k)[:0] for k in ("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg",
                                                                  "t_slen")})
    res = sw.run(e.sw_input(), sw.default_opts(finish=False))
    assert len(res["status"]) == 0


@pytest.mark.gpu
def test_sw_gpu_rejects_reads_beyond_proovread_limit():
    from proovread_amd import sw, synth
    d = synth.simulate(4, 20000, 4, 3000, 3.0, sr_len=1001)
    with pytest.raises(RuntimeError, match="longer than 1000"):
        sw.run(d.sw_input(), sw.default_opts(finish=False))


@pytest.mark.gpu
@pytest.mark.parametrize("task", ["bwa-sr", "bwa-sr-finish"])
def test_sw_gpu_cigar_overflow_pass(task, monkeypatch):
    """Every slot forced to 16 ops (PRGPU_SW_CIG_SLOT): most CIGARs outgrow their slot and go
    through the overflow pass (spill area, general kernel); results stay bit-exact."""
    from proovread_amd import sw, synth
    monkeypatch.setenv("PRGPU_SW_CIG_SLOT", "16")
    d = synth.simulate(8, 60000, 20, 3000, 10.0, sr_frac=1.0)
    res = sw.run(d.sw_input(), sw.default_opts(finish=task.endswith("finish")))
    assert (res["status"] == 0).all()
    assert res.n_overflow > len(d.t_sr) // 4
    idx = np.arange(0, len(d.t_sr), max(1, len(d.t_sr) // 400))
    want = oracle_results(d, ob.sw_opts(task), idx)
    bad = [(int(t), w, gpu_tuple(res, t)) for t, w in zip(idx, want) if tuple(w) != gpu_tuple(res, t)]
    assert not bad, bad[:3]
