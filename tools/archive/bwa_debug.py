"""Debug driver for bwa mode on the device: one small synthetic batch through pr_sw_run
with progress on stderr (PRGPU_BWA_DEBUG), then the oracle comparison read by read."""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))
os.environ.setdefault("PRGPU_BWA_DEBUG", "1")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    from proovread_amd import _abi, seed, sw, synth
    finish = len(sys.argv) > 1 and sys.argv[1] == "finish"
    d = synth.simulate(41, 40000, 40, 2500, 15)
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    d = synth.with_seeds(d, ix.map(d.sr_seq, d.sr_off, seed.default_opts(finish), threads=4))
    log("seeds", len(d.t_sr), "reads", d.n_sr)
    ctx = _abi.default_context()
    t = time.time()
    res = sw.run(d.sw_input(), sw.default_opts(finish), ctx=ctx)
    log("sw.run", time.time() - t, "alignments", res.n, "stats", sw.bwa_stats(ctx))
    import cpu_chain
    want = cpu_chain.bwa_alignments(d, "bwa-sr-finish" if finish else "bwa-sr")
    got = {}
    for i in range(res.n):
        tk = int(res["task"][i])
        got.setdefault(int(d.t_sr[tk]), []).append(
            (int(d.t_lr[tk]), int(d.t_strand[tk]), int(res["pos"][i]), [int(x) for x in res.cigar_ops(i)],
             int(res["score"][i]), int(res["flag"][i]), int(res["qb"][i]), int(res["qe"][i]), int(res["rb"][i]),
             int(res["re"][i]), int(res["truesc"][i]), tk))
    bad = [r for r in range(d.n_sr) if got.get(r, []) != want[r]]
    log("reads differing", len(bad), "of", d.n_sr)
    for r in bad[:3]:
        log("read", r, "\n got ", got.get(r), "\n want", want[r])


if __name__ == "__main__":
    main()
