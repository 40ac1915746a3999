"""Time the GPU seeding path alone on the bench's configs[1] workload (index build + map),
with its phase counters; PRGPU_SEED_WAVES_PER_CU tunes pass 1's grid."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from proovread_amd import _abi, seed, synth
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    d = synth.simulate(20261015 + 2, int(4_600_000 * scale), int(13_800 * scale), 10_000, 50.0, sr_frac=0.3)
    ctx = _abi.Context(0)
    ix = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
    o = seed.default_opts(False)
    for rep in range(2):
        t = time.perf_counter()
        tasks, _ = ix.map(d.sr_seq, d.sr_off, o)
        wall = time.perf_counter() - t
    print(json.dumps({"waves_per_cu": os.environ.get("PRGPU_SEED_WAVES_PER_CU"), "reads": d.n_sr, "index_ms": round(ix.build_ms(), 1),
                      "seeds": int(len(tasks)), "kernel_ms": round(ix.gpu_ms(), 1), "map_wall_s": round(wall, 3),
                      "phases": ix.phase_ms()}), flush=True)


if __name__ == "__main__":
    main()
