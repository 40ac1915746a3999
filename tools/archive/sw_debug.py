"""GPU debugging aid: run the SW stage on the clr15 test dataset and print the
first mismatches against the oracle in full (fields and CIGAR strings)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import oracle_bind as ob  # noqa: E402
from sw_util import gpu_tuple, oracle_results, with_ns  # noqa: E402
from proovread_amd import sw, synth  # noqa: E402

d = synth.simulate(11, 60000, 200, 3000, 20)
d = with_ns(d, np.random.default_rng(3))
opts = sw.default_opts(finish=False)
res = sw.run(d.sw_input(), opts)
idx = np.arange(0, len(d.t_sr), 7)[:4000]
want = oracle_results(d, ob.sw_opts("bwa-sr"), idx)
bad = [(int(t), w, gpu_tuple(res, t)) for t, w in zip(idx, want) if tuple(w) != gpu_tuple(res, t)]
print("checked", len(idx), "bad", len(bad))
for t, w, g in bad[:6]:
    print("task", t, "strand", int(d.t_strand[t]))
    print("  want", w)
    print("  got ", g)
