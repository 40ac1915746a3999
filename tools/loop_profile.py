"""Host vs device time of the correction loop (correct.run with the GPU stages) on a configs[1]-size
input (GPU box): per task the wall time, the device time the library's HIP events report (index
build, seeding, SW + hand-off + consensus, masking) and the host remainder; plus a cProfile of
the host side.

    python tools/loop_profile.py [scale] [out.json]
"""
import cProfile
import io
import json
import pstats
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from proovread_amd import correct, synth  # noqa: E402

ACGT = np.frombuffer(b"ACGTN", np.uint8)


def fastq_bytes(seq, off):
    """FASTQ records @sr<i> of equal-length reads, built with numpy."""
    n = len(off) - 1
    L = int(off[1] - off[0])
    assert (np.diff(off) == L).all()
    seq = seq[:int(off[-1])]
    heads = [b"@sr%d\n" % i for i in range(n)]
    hl = np.array([len(h) for h in heads], np.int64)
    rec = hl + L + 1 + 2 + L + 1
    ro = np.zeros(n + 1, np.int64)
    np.cumsum(rec, out=ro[1:])
    buf = np.empty(int(ro[-1]), np.uint8)
    hb = np.frombuffer(b"".join(heads), np.uint8)
    ho = np.zeros(n + 1, np.int64)
    np.cumsum(hl, out=ho[1:])
    # head bytes
    idx = np.repeat(ro[:-1] - ho[:-1], hl) + np.arange(int(ho[-1]))
    buf[idx] = hb
    base = ro[:-1] + hl
    s = ACGT[seq].reshape(n, L)
    cols = np.arange(L)
    buf[(base[:, None] + cols[None, :]).reshape(-1)] = s.reshape(-1)
    buf[base + L] = 10
    buf[base + L + 1] = ord("+")
    buf[base + L + 2] = 10
    buf[((base + L + 3)[:, None] + cols[None, :]).reshape(-1)] = ord("I")
    buf[base + 2 * L + 3] = 10
    return buf.tobytes()


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    out = sys.argv[2] if len(sys.argv) > 2 else None
    t = time.perf_counter()
    # the bench's dataset: short reads in sequencer order (unsorted over the genome), as a FASTQ
    # from a sequencing run is -- SeqChunker's contiguous chunks then sample the whole genome
    gl = int(4_600_000 * scale)
    d = synth.simulate_reads(20261015 + 2, gl, int(13_800 * scale), 10_000, int(round(50.0 * gl / 150)), threads=16)
    lrs = [(f"lr{i}", ACGT[d.lr_seq[d.lr_off[i]:d.lr_off[i + 1]]].tobytes(), None) for i in range(d.n_lr)]
    srd = fastq_bytes(d.sr_seq, d.sr_off)
    gen_s = time.perf_counter() - t
    print(f"generated {d.n_lr} long reads, {d.n_sr} short reads ({len(srd) / 1e6:.0f} MB FASTQ) in {gen_s:.1f} s",
          flush=True)
    cfg = correct.LoopConfig(coverage=50.0)
    stages = correct.GpuStages()
    prof = cProfile.Profile()
    t = time.perf_counter()
    prof.enable()
    res = correct.run(lrs, srd, cfg, stages=stages)
    prof.disable()
    wall = time.perf_counter() - t
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(40)
    rows = [{"task": e.task, "n_sr": e.n_sr, "n_tasks": e.n_tasks, "wall_ms": e.wall_ms, "device_ms": e.device_ms,
             "host_ms": (round(e.wall_ms - e.device_ms, 1) if e.wall_ms is not None and e.device_ms is not None
                         else None), "masked_frac": e.masked_frac, "shortcut": e.shortcut} for e in res.log]
    summary = {"scale": scale, "long_reads": d.n_lr, "short_reads": d.n_sr, "loop_wall_s": round(wall, 2),
               "tasks": rows}
    print(json.dumps(summary, indent=1))
    print(s.getvalue())
    if out:
        Path(out).write_text(json.dumps(summary, indent=1) + "\n")


if __name__ == "__main__":
    main()
