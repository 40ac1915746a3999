"""One timed `bwa-proovread mem` run on configs[1]'s bwa-sr-1 sample, the
way bin/proovread:1313 runs it: the long reads as FASTA, the task's short-read sample as FASTQ
(SeqChunker's chunks of the 50x run in sequencer order), bwa-sr-1's options with -b 20 -l 300,
SAM on stdout (here /dev/null, as proovread pipes it into `samtools view`).  Prints the wall time
of the process and its own stage log.

    python tools/time_mem_dropin.py [out.json]
"""
import json
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))


def main():
    from proovread_amd import control, correct, synth
    from proovread_amd import tasks as T
    from loop_profile import fastq_bytes
    gl, n_lr = 4_600_000, 13_800
    d = synth.simulate_reads(20261015 + 2, gl, n_lr, 10_000, int(round(50.0 * gl / 150)), threads=16)
    srs = correct.ShortReads.from_pool(d.sr_seq[:int(d.sr_off[-1])], d.sr_off)
    rg, off = srs.sample_ranges(control.Sampler().cov2seqchunker(50.0, T.sr_coverage("bwa-sr-1")))
    seq = srs.gather(rg)
    asc = np.frombuffer(b"ACGTN", np.uint8)
    with tempfile.TemporaryDirectory(prefix="memdrop_") as td:
        lr_fa, sr_fq = Path(td) / "lr.fa", Path(td) / "sr.fq"
        with open(lr_fa, "wb") as fh:
            for i in range(n_lr):
                fh.write(b">lr%d\n" % i)
                fh.write(asc[d.lr_seq[d.lr_off[i]:d.lr_off[i + 1]]].tobytes() + b"\n")
        sr_fq.write_bytes(fastq_bytes(seq, off))
        argv = ["-b", "20", "-l", "300"] + T.bwa_argv("bwa-sr-1") + ["-t", "16", str(lr_fa), str(sr_fq)]
        t = time.perf_counter()
        with open("/dev/null", "w") as sink:
            r = subprocess.run([sys.executable, "-m", "proovread_amd.bwa_proovread", "mem", *argv], stdout=sink,
                               stderr=subprocess.PIPE, text=True, cwd=ROOT)
        wall = time.perf_counter() - t
    rec = {"short_reads": int(len(off) - 1), "long_reads": n_lr, "wall_s": round(wall, 2), "rc": r.returncode,
           "log": r.stderr.strip().splitlines()[-6:]}
    print(json.dumps(rec, indent=1))
    if len(sys.argv) > 1:
        Path(sys.argv[1]).write_text(json.dumps(rec, indent=1) + "\n")
    if r.returncode:
        sys.exit(r.returncode)


if __name__ == "__main__":
    main()
