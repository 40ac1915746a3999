"""GPU seeding in the finish task's setting: the short reads mapped to CORRECTED long reads
(near-exact, 30x long-read coverage: every 12-mer of a read hits ~30 copies) with the
bwa-sr-finish options; configs[1] size.  Prints the kernel time and how many reads pass 1's
slices could not hold (pass 2: one wave per read)."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from proovread_amd import _abi, seed, synth
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    d = synth.simulate(20261015 + 2, int(4_600_000 * scale), int(13_800 * scale), 10_000, 50.0, p_ins=0.002,
                       p_del=0.002, p_sub=0.002, sr_frac=0.6)
    ctx = _abi.Context(0)
    ix = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
    o = seed.default_opts(True)
    for rep in range(2):
        t = time.perf_counter()
        tasks, st = ix.map(d.sr_seq, d.sr_off, o, allow_flagged=True)
        wall = time.perf_counter() - t
    print(json.dumps({"reads": int(d.n_sr), "flagged": int((st != 0).sum()), "seeds": int(len(tasks)),
                      "index_ms": round(ix.build_ms(), 1), "kernel_ms": round(ix.gpu_ms(), 1),
                      "map_wall_s": round(wall, 3), "phases": ix.phase_ms()}), flush=True)


if __name__ == "__main__":
    main()
