"""time GPU seeding in mr mode, where mem_flt_chained_seeds' local SW
(seed_core.h seed_sw_score: a scalar DP over H / E rows in the lane's scratch) runs for every
seed of every kept chain of reads >= 440 bp.  Reads of 300 (below the threshold: no filter),
600 and 950 bases against 10 kb long reads at 15 % error; the bwa-mr-1 seeding options.
Prints the GPU kernel time, the pass-1 lane split (PRGPU_SEED_DEBUG: SMEMs / chaining / filter +
output, summed over lanes) and the seeds per read.

    PRGPU_SEED_DEBUG=1 python tools/seed_time_mr.py > out.log
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from proovread_amd import _abi, seed, synth, tasks as T
    ctx = _abi.Context(0)
    for sr_len in (300, 600, 950):
        d = synth.simulate(20261017 + sr_len, 1_000_000, 3_000, 10_000, 15.0, sr_len=sr_len, sr_frac=1.0)
        ix = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
        o = T.options("bwa-mr-1")[0]
        for rep in range(2):
            t = time.perf_counter()
            tasks, st = ix.map(d.sr_seq, d.sr_off, o, allow_flagged=True)
            wall = time.perf_counter() - t
        print(json.dumps({"sr_len": sr_len, "reads": int(d.n_sr), "flagged": int((st != 0).sum()),
                          "seeds": int(len(tasks)), "seeds_per_read": round(len(tasks) / d.n_sr, 1),
                          "kernel_ms": round(ix.gpu_ms(), 1), "map_wall_s": round(wall, 3),
                          "phases": ix.phase_ms()}), flush=True)


if __name__ == "__main__":
    main()
