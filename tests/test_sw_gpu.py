"""GPU parity of the seed-extension stage (libprgpu.so via the C-ABI) against
the SW oracle (oracle/sw_oracle.c, restatement of upstream bwa ksw/mem; parity
against bwa-proovread itself is unpinned).

Bar: bit-exact qb/qe/rb/re, AS (score), truesc, POS, CIGAR and -T pass flag
for every task, on seeded synthetic inputs covering both strands, seeds at
read starts/ends, N bases in the long reads, the iteration and the finish
scoring schemes, and 25 kb / 20 %-error long reads (config 5 style).
"""
import numpy as np
import pytest

import oracle_bind as ob
from sw_util import gpu_tuple, oracle_results, with_ns

pytestmark = pytest.mark.gpu


def _compare(d, task="bwa-sr", n_check=3000, seed=0):
    from proovread_amd import sw
    opts = sw.default_opts(finish=(task == "bwa-sr-finish"))
    res = sw.run(d.sw_input(), opts)
    assert (res["status"] == 0).all()
    rng = np.random.default_rng(seed)
    n = len(d.t_sr)
    idx = np.unique(np.concatenate([rng.choice(n, size=min(n_check, n), replace=False),
                                    np.nonzero(d.t_qbeg == 0)[0][:50],
                                    np.nonzero(d.t_qbeg + d.t_slen == 150)[0][:50]]))
    want = oracle_results(d, ob.sw_opts(task), idx)
    bad = [(int(t), w, gpu_tuple(res, t)) for t, w in zip(idx, want) if tuple(w) != gpu_tuple(res, t)]
    assert not bad, bad[:3]
    return res


@pytest.mark.parametrize("task", ["bwa-sr", "bwa-sr-finish"])
def test_sw_gpu_matches_oracle_clr15(task):
    from proovread_amd import synth
    d = synth.simulate(11, 60000, 200, 3000, 20)
    d = with_ns(d, np.random.default_rng(3))
    _compare(d, task)


def test_sw_gpu_matches_oracle_high_error_25kb():
    from proovread_amd import synth
    d = synth.simulate(12, 200000, 12, 25000, 10, p_ins=0.05, p_del=0.08, p_sub=0.07)
    _compare(d, "bwa-sr", n_check=1500)


def test_sw_gpu_cell_count_and_timing():
    from proovread_amd import _abi, sw, synth
    d = synth.simulate(13, 30000, 60, 2000, 10)
    ctx = _abi.default_context()
    sw.run(d.sw_input(), ctx=ctx)
    ms_e, ms_g, ce, cg = sw.last_timing(ctx)
    assert ms_e > 0 and ms_g > 0
    # at least one extension side of ~q*(2w+1) cells per task on average
    assert ce > len(d.t_sr) * 1000 and cg > len(d.t_sr) * 100
