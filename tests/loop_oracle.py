"""CPU stages for proovread_amd.correct's loop (TEST INFRASTRUCTURE ONLY).

Same interface as correct.GpuStages, computed by the oracles: the SW oracle ->
SAM order -> consensus oracle chain (oracle/cpu_chain.py) for an iteration, and
the mask_hcrs restatement (oracle/seqfilter_oracle.py) for SeqFilter
--phred-mask.  The GPU loop must reproduce this loop byte-for-byte."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import cpu_chain  # noqa: E402
import seqfilter_oracle as SO  # noqa: E402


class OracleStages:
    def __init__(self, workers: int = 4):
        self.workers = workers

    def iteration(self, d, ref_seq, ref_qual, task, params, bin_filter=None):
        from proovread_amd import tasks as T
        o = T.options(task)[1]
        sw = (o.a, o.b, o.o_del, o.o_ins, o.e_del, o.e_ins, o.w, o.pen_clip5, o.pen_clip3, o.zdrop,
              o.min_score_per_base)
        _, _, res, _ = cpu_chain.run_sample(
            d, range(d.n_lr), task=sw, coverage=params.coverage,
            use_ref_qual=params.use_ref_qual, workers=self.workers, ref_seq=ref_seq, ref_qual=ref_qual,
            detect_chimera=params.detect_chimera, full=True, bin_filter=bin_filter)
        out = []
        for rc, fq, _trace, chim in res:
            if rc:
                out.append((rc, b"", b"", []))
                continue
            lines = fq.split("\n")
            out.append((0, lines[1].encode("latin-1"), lines[3].encode("latin-1"),
                        [ln for ln in chim.split("\n") if ln]))
        return out

    def mask(self, seqs, quals, hcr_mask, min_sr_length):
        masked, _, (bpt, bpn) = SO.mask_reads(seqs, quals, SO.mask_params_from_cfg(hcr_mask, min_sr_length))
        return masked, bpt, bpn
