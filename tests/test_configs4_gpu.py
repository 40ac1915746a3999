"""BASELINE configs[4] shape on the GPU: 25 kb long reads at 20 %
error (5 % insertions, 8 % deletions, 7 % substitutions), the band override -w 100
(first extension try at w = 100, the second at 200: the wide-band extension kernel and
the general CIGAR kernel), and the deep pileup of `--coverage 100` with sr-coverage 50
(consensus cap 37.5).  Bar: the SW outputs bit-exact against the SW oracle, and one whole
iteration (SW -> hand-off -> consensus) byte-exact against the CPU chain."""
import numpy as np
import pytest

import oracle_bind as ob
from sw_util import gpu_tuple, oracle_results

pytestmark = pytest.mark.gpu


def _data(seed, n_lr=5, sr_cov=30.0):
    from proovread_amd import synth
    return synth.simulate(seed, 50_000, n_lr, 25_000, sr_cov, p_ins=0.05, p_del=0.08, p_sub=0.07, sr_frac=1.0)


def _opts(task, w):
    from proovread_amd import sw
    o = sw.default_opts(finish=task.endswith("finish"))
    o.w = w
    so = ob.sw_opts(task)
    so.w = w
    return o, so


@pytest.mark.parametrize("task", ["bwa-sr", "bwa-sr-finish"])
def test_sw_wide_band_matches_oracle(task):
    from proovread_amd import sw
    d = _data(41, n_lr=3, sr_cov=10.0)
    o, so = _opts(task, 100)
    res = sw.run(d.sw_input(), o)
    assert (res["status"] == 0).all()
    idx = np.arange(0, len(d.t_sr), max(1, len(d.t_sr) // 300))
    want = oracle_results(d, so, idx)
    bad = [(int(t), w, gpu_tuple(res, t)) for t, w in zip(idx, want) if tuple(w) != gpu_tuple(res, t)]
    assert not bad, bad[:3]


def test_iteration_configs4_matches_cpu_chain():
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
    import cpu_chain
    from proovread_amd import cns, iteration
    d = _data(43)
    o, so = _opts("bwa-sr", 100)
    it = iteration.Iteration(d)
    it.launch(o, cns.CnsParams(coverage=37.5, use_ref_qual=True))
    got = it.results()
    swt = (so.a, so.b, so.o_del, so.o_ins, so.e_del, so.e_ins, so.w, so.pen_clip5, so.pen_clip3, so.zdrop,
           so.min_score_per_base)
    _, _, want, _ = cpu_chain.run_sample(d, range(d.n_lr), task=swt, coverage=37.5, use_ref_qual=True, workers=8,
                                         full=True)
    for i, (g, w) in enumerate(zip(got, want)):
        rc, fq, tr, _ = w
        assert rc == 0 and g.status == 0, (i, rc, g.status)
        assert g.fastq == fq, i
        assert g.trace == tr, i
