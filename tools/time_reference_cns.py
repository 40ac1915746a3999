"""Time the reference's own CPU consensus path (the Perl Sam::Seq engine of bam2cns, run by
tests/golden/gen_cns_golden.pl) beside the C oracle on the same long reads of the bench
workload (configs[1] parameters: 10 kb CLR reads, 15x short reads, coverage cap 11.25,
reference qualities on).  Needs /root/reference (build container only); writes a JSON
summary (profiles/r01_reference_cpu_consensus.json).

    python tools/time_reference_cns.py [n_long_reads] [out.json]
"""
import ctypes as C
import json
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tests" / "golden"), str(ROOT / "oracle")]
import oracle_bind as ob  # noqa: E402
from casefmt import Case, write_cases  # noqa: E402

from proovread_amd import synth  # noqa: E402

ASCII = np.frombuffer(b"ACGTN", np.uint8)


def main():
    n_lr = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    out = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "profiles" / "r01_reference_cpu_consensus.json"
    d = synth.simulate(20261017, 400_000, 1200, 10_000, 50.0, sr_frac=0.3)   # 30x LR, 15x SR, like configs[1]
    off = np.zeros(d.n_lr + 1, np.int64)
    np.cumsum(np.bincount(d.t_lr, minlength=d.n_lr), out=off[1:])
    L = ob.sw_lib()
    opts = ob.sw_opts("bwa-sr")
    r = ob.OswResult()
    cases = []
    for lr in range(n_lr):
        Llen = int(d.lr_off[lr + 1] - d.lr_off[lr])
        recs = []
        for t in range(int(off[lr]), int(off[lr + 1])):
            sid = int(d.t_sr[t])
            so, lq = int(d.sr_off[sid]), int(d.sr_off[sid + 1] - d.sr_off[sid])
            rc = L.osw_task(C.byref(opts), C.cast(d.sr_seq.ctypes.data + so, C.POINTER(C.c_uint8)), lq,
                            C.cast(d.lr_seq.ctypes.data + int(d.lr_off[lr]), C.POINTER(C.c_uint8)), Llen,
                            int(d.t_strand[t]), int(d.t_qbeg[t]), int(d.t_rbeg[t]), int(d.t_slen[t]), C.byref(r))
            if rc or not getattr(r, "pass"):
                continue
            st = int(d.t_strand[t])
            q = d.sr_seq[so:so + lq]
            s = (ASCII[np.where(q < 4, 3 - q, 4)][::-1] if st else ASCII[q]).tobytes().decode()
            cg = "".join(f"{x >> 4}{'MIDNSHP=X'[x & 15]}" for x in r.cigar[:r.n_cigar])
            recs.append((r.pos, st, t, f"sr{sid}\t{16 if st else 0}\tlr{lr}\t{r.pos + 1}\t60\t{cg}\t*\t0\t0\t{s}\t*\t"
                                       f"AS:i:{r.score}"))
        recs.sort(key=lambda x: (x[0], x[1], x[2]))
        ref = ASCII[d.lr_seq[int(d.lr_off[lr]):int(d.lr_off[lr + 1])]].tobytes().decode()
        cases.append(Case(f"lr{lr}", {"coverage": "11.25", "use_ref_qual": "1"}, [f"@lr{lr}", ref, "+", "$" * Llen],
                          [x[3] for x in recs]))
    cols = sum(len(c.ref[1]) for c in cases)
    alns = sum(len(c.sam) for c in cases)
    with tempfile.TemporaryDirectory() as td:
        cf = Path(td) / "cases.txt"
        write_cases(cf, cases)
        t = time.perf_counter()
        perl = subprocess.run(["perl", str(ROOT / "tests" / "golden" / "gen_cns_golden.pl"), str(cf)],
                              capture_output=True, text=True, env={"PERL_HASH_SEED": "0", "PERL_PERTURB_KEYS": "0",
                                                                   "PATH": "/usr/bin:/bin"}, check=True)
        t_perl = time.perf_counter() - t
        ef = Path(td) / "expected.txt"
        ef.write_text(perl.stdout)
        from casefmt import read_expect
        expect = read_expect(ef)
    t = time.perf_counter()
    res = [ob.run_case(c) for c in cases]
    t_c = time.perf_counter() - t
    ok = sum(1 for x in res if x["rc"] == 0)
    same = sum(1 for c, x in zip(cases, res)
               if x["rc"] == 0 and not expect[c.name].error and x["fastq"].rstrip("\n").split("\n") == expect[c.name].fastq
               and x["trace"] == expect[c.name].trace and x["kept"] == expect[c.name].kept)
    summary = {
        "what": "consensus of long reads of the bench workload (configs[1] parameters), one CPU core each",
        "long_reads": n_lr, "columns": cols, "alignments": alns,
        "reference_perl": {"engine": "lib/Sam/Seq.pm via tests/golden/gen_cns_golden.pl (bam2cns per-read loop)",
                           "seconds": round(t_perl, 3), "columns_per_s": round(cols / t_perl, 1),
                           "Mbases_per_s": round(cols / t_perl / 1e6, 5), "cores": 1},
        "oracle_c": {"seconds": round(t_c, 3), "columns_per_s": round(cols / t_c, 1), "cores": 1, "ok": ok,
                     "reads_identical_to_perl": same},
        "host": "build container, 8 vCPU",
    }
    out.write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary))
    assert perl.stdout.count(">>CASE") == n_lr


if __name__ == "__main__":
    main()
