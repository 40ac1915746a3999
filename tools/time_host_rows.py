"""Host-side throughput of the §8f rows that run on the CPU (build container, 8 vCPU):
seeding front end (pr_seed_map, and its index build), BAM I/O (SAM -> BAM, coordinate sort,
BAI index: the samtools drop-in), final trim windows (pr_trim_windows), SeqChunker sampling.
Synthetic inputs of configs[1] shape.  Writes profiles/r01_host_rows.json.

    python tools/time_host_rows.py [out.json]
"""
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from proovread_amd import bamio, seed, seqchunker, synth, trim  # noqa: E402


def main():
    out = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "profiles" / "r01_host_rows.json"
    res = {"host": "build container, 8 vCPU", "threads": 8}
    d = synth.simulate(20261017, 4_600_000, 13_800, 10_000, 50.0, sr_frac=0.3)   # configs[1]
    t = time.perf_counter()
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    t_ix = time.perf_counter() - t
    n = 100_000
    so = d.sr_off[:n + 1]
    t = time.perf_counter()
    tasks = ix.map(d.sr_seq[:so[-1]], so, threads=8)
    t_map = time.perf_counter() - t
    ix.close()
    res["seeding_host"] = {"index_build_s": round(t_ix, 2), "long_read_bases": int(d.lr_off[-1]),
                           "reads": n, "map_s": round(t_map, 2), "reads_per_s": round(n / t_map, 1),
                           "tasks": int(len(tasks)),
                           "iteration_reads_configs1": int(d.n_sr),
                           "iteration_map_s_est": round(d.n_sr / (n / t_map), 1)}
    # BAM I/O: 400k records against 2000 long reads
    rng = np.random.default_rng(1)
    nrec, nref = 400_000, 2000
    names = [f"lr{i}" for i in range(nref)]
    header = "@HD\tVN:1.5\tSO:unsorted\n" + "".join(f"@SQ\tSN:{x}\tLN:10000\n" for x in names)
    seq150 = "ACGT" * 37 + "AC"
    lines = [f"sr{k}\t{16 if k & 1 else 0}\t{names[int(rng.integers(nref))]}\t{int(rng.integers(1, 9800))}\t60\t"
             f"150M\t*\t0\t0\t{seq150}\t*\tAS:i:{int(rng.integers(300, 750))}" for k in range(nrec)]
    with tempfile.TemporaryDirectory() as td:
        p_u, p_s = str(Path(td) / "u.bam"), str(Path(td) / "s.bam")
        t = time.perf_counter()
        bamio.write_bam_from_sam(iter(lines), p_u, header)
        t_w = time.perf_counter() - t
        t = time.perf_counter()
        bamio.sort_bam(p_u, p_s)
        t_s = time.perf_counter() - t
        t = time.perf_counter()
        bamio.index_bam(p_s)
        t_i = time.perf_counter() - t
        t = time.perf_counter()
        m = sum(1 for _ in bamio.region_records(p_s, names[7]))
        t_q = time.perf_counter() - t
        size = Path(p_s).stat().st_size
    res["bam_io"] = {"records": nrec, "sam_to_bam_s": round(t_w, 2), "sort_s": round(t_s, 2), "index_s": round(t_i, 2),
                     "records_per_s_write": round(nrec / t_w, 1), "records_per_s_sort": round(nrec / t_s, 1),
                     "region_query_ms": round(t_q * 1e3, 2), "region_records": m, "bam_bytes": size}
    # trim windows over 2000 x 10 kb reads with mixed qualities
    quals = []
    for _ in range(2000):
        ph, hi = [], True
        while len(ph) < 10_000:
            k = int(rng.integers(20, 2000))
            ph += list(rng.integers(20, 41, k) if hi else rng.integers(0, 15, k))
            hi = not hi
        quals.append(bytes(33 + x for x in ph[:10_000]))
    p = trim.params("12,5")
    t = time.perf_counter()
    w = trim.windows(quals, p, threads=8)
    t_t = time.perf_counter() - t
    res["trim_windows"] = {"reads": len(quals), "bases": 2000 * 10_000, "s": round(t_t, 3),
                           "Mbases_per_s": round(2e7 / t_t / 1e6, 1), "windows": int(sum(len(x) for x in w))}
    # SeqChunker over a FASTQ of 200k short reads
    fq = b"".join(b"@r%d\n%s\n+\n%s\n" % (i, b"A" * 150, b"I" * 150) for i in range(200_000))
    t = time.perf_counter()
    nch, chunks = seqchunker.chunk(fq, 1000)
    sel = seqchunker.select(nch, 1, 20, 6)
    blob = b"".join(fq[s:e] for k in sel for s, e in chunks[k - 1])
    t_c = time.perf_counter() - t
    res["seqchunker"] = {"bytes": len(fq), "s": round(t_c, 3), "MB_per_s": round(len(fq) / t_c / 1e6, 1),
                         "selected_fraction": round(len(blob) / len(fq), 3)}
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
