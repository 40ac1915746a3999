"""The oracle chain's worker pool never forks a process that holds a HIP runtime (VERDICT r05
item 6: a forked child of a GPU test process segfaulted and the old fork pool replaced it
silently).  With HIP loaded, oracle/cpu_chain.run_sample runs in a fresh child process whose
own pool forks; a worker that dies breaks the pool (BrokenProcessPool) instead of being
replaced.  CPU only: the HIP check is forced here."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))


def _data():
    from proovread_amd import seed, synth
    d = synth.simulate(41, 30_000, 12, 3_000, 20)
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    try:
        return synth.with_seeds(d, ix.map(d.sr_seq, d.sr_off, seed.default_opts(False), threads=2))
    finally:
        ix.close()


def test_child_process_equals_in_process(monkeypatch):
    import cpu_chain
    d = _data()
    kw = dict(coverage=11.25, use_ref_qual=True, workers=2, full=True, bin_filter=(20, 300.0))
    _, b0, want, _ = cpu_chain.run_sample(d, range(d.n_lr), **kw)
    monkeypatch.setattr(cpu_chain, "_hip_in_process", lambda: True)
    _, b1, got, _ = cpu_chain.run_sample(d, range(d.n_lr), **kw)
    assert b0 == b1 and got == want and all(r[0] == 0 for r in want)
    # SAM lines (sam_only) come back as lists
    _, _, sam_want, _ = cpu_chain.run_sample(d, range(3), workers=2, sam_only=True, bin_filter=(20, 300.0))
    monkeypatch.setattr(cpu_chain, "_hip_in_process", lambda: False)
    _, _, sam_in, _ = cpu_chain.run_sample(d, range(3), workers=2, sam_only=True, bin_filter=(20, 300.0))
    assert sam_want == sam_in and sum(len(x) for x in sam_in) > 0


def _die(x):
    import os
    if x == 3:
        os._exit(11)
    return x


def test_dead_worker_fails_loudly():
    import cpu_chain
    from concurrent.futures.process import BrokenProcessPool
    with pytest.raises(BrokenProcessPool):
        cpu_chain._pool_map(_die, list(range(8)), 2, 1)
