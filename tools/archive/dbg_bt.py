"""Debug: SW CIGAR pass vs the oracle on the clr15 dataset of tests/test_sw_gpu.py, printing
the first differing tasks in full (PRGPU_SW_DEBUG=8 disables the bulk I-run backtrack)."""
import sys
sys.path[:0] = ["/root/repo", "/root/repo/tests", "/root/repo/tests/golden"]
import numpy as np
import oracle_bind as ob
from proovread_amd import sw, synth
from sw_util import gpu_tuple, oracle_results, with_ns
d = with_ns(synth.simulate(11, 60000, 200, 3000, 20), np.random.default_rng(3))
res = sw.run(d.sw_input(), sw.default_opts(finish=False))
idx = np.arange(0, len(d.t_sr), max(1, len(d.t_sr) // 2000))
want = oracle_results(d, ob.sw_opts("bwa-sr"), idx)
bad = [(int(t), tuple(w), gpu_tuple(res, t)) for t, w in zip(idx, want) if tuple(w) != gpu_tuple(res, t)]
print("checked", len(idx), "bad", len(bad))
for b in bad[:6]:
    print(b[0]); print("  want", b[1]); print("  got ", b[2])
