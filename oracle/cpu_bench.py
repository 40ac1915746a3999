"""ORACLE — BASELINE / CHECKER ONLY (bench.py's cpu_baseline leg, run as a child process).

Loads the bench workload bench.py saved (reads + seeds, .npz; bwa mode when t_chain is
there: the seeds of every short read with a seed on the first N long reads), runs the
CPU chain (oracle/cpu_chain.py: bwa mem per-read alignment restatement -> SAM order ->
consensus restatement) on the first N long reads over W worker processes, and writes one JSON object: the
timing and, per read, (rc, fastq, trace, chim lines) for bench.py's byte-for-byte
comparison with the GPU output.  A separate process, so the fork pool never shares a
process with a HIP runtime.

    python oracle/cpu_bench.py WORKLOAD.npz N WORKERS OUT.json [finish [BIN LEN]]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))


def main(argv) -> int:
    path, n, workers, out = argv[0], int(argv[1]), int(argv[2]), argv[3]
    finish = len(argv) > 4 and argv[4] == "1"
    binf = (int(argv[5]), float(argv[6])) if len(argv) > 6 else None
    z = np.load(path)   # allow_pickle=False: arrays only
    d = SimpleNamespace(**{k: z[k] for k in z.files})
    d.n_lr = len(d.lr_off) - 1
    d.n_sr = len(d.sr_off) - 1
    if "t_chain" not in z.files:
        d.t_chain = None
    import cpu_chain
    n = min(n, d.n_lr)
    wall, bases, res, nw = cpu_chain.run_sample(d, range(n), task="bwa-sr-finish" if finish else "bwa-sr",
                                                coverage=22.5 if finish else 11.25, use_ref_qual=not finish,
                                                detect_chimera=finish, workers=workers, full=True, bin_filter=binf)
    with open(out, "w") as f:
        json.dump({"wall_s": wall, "bases": bases, "workers": nw, "n": n,
                   "tasks": int(len(d.t_sr)) if d.t_chain is not None else int(np.searchsorted(d.t_lr, n, side="left")),
                   "results": [list(r) for r in res]}, f)
    return 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1:]))
