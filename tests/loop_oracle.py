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
            detect_chimera=params.detect_chimera, full=True, bin_filter=bin_filter, drop_ratio=o.drop_ratio)
        return self._out(res)

    @staticmethod
    def _out(res):
        out = []
        for rc, fq, _trace, chim in res:
            if rc:
                out.append((rc, b"", b"", []))
                continue
            lines = fq.split("\n")
            out.append((0, lines[1].encode("latin-1"), lines[3].encode("latin-1"),
                        [ln for ln in chim.split("\n") if ln]))
        return out

    def align(self, d, task):
        """bwa-mode alignments of d's seeds (aln_oracle.c), SAM order, read by read:
        (sr, lr, strand, pos, score, flag, cigar ops)."""
        from proovread_amd import tasks as T
        o = T.options(task)[1]
        sw = (o.a, o.b, o.o_del, o.o_ins, o.e_del, o.e_ins, o.w, o.pen_clip5, o.pen_clip3, o.zdrop,
              o.min_score_per_base)
        reads = sorted(set(int(x) for x in d.t_sr))
        per = cpu_chain.bwa_alignments(d, sw, drop_ratio=o.drop_ratio, reads=reads)
        return [(r, a[0], a[1], a[2], a[4], a[5], a[3]) for r, v in zip(reads, per) for a in v]

    def consensus(self, ids, ref_seq, ref_qual, sams, params):
        """The consensus oracle on SAM lines already in samtools order."""
        import ctypes as C
        import oracle_bind as ob
        P = ob.OcnsParams()
        P.max_coverage, P.bin_size, P.trim, P.indel_taboo_length, P.indel_taboo = params.coverage, 20.0, 1, 7, 0.1
        P.min_aln_length, P.max_ins_length, P.fallback_phred, P.phred_offset, P.ref_phred_offset = 50, 0, 1, 33, 33
        P.use_ref_qual, P.qual_weighted, P.detect_chimera, P.invert_scores = int(params.use_ref_qual), 0, \
            int(params.detect_chimera), 0
        res = []
        for i, lines in enumerate(sams):
            enc = [x.encode() for x in lines]
            arr = (C.c_char_p * (len(enc) + 1))(*enc)
            r = ob.OcnsResult()
            rc = ob.lib().ocns_run(C.byref(P), ids[i].encode(), ref_seq[i], ref_qual[i], len(ref_seq[i]), arr,
                                   len(enc), None, 0, C.byref(r))
            res.append((rc, r.fastq.decode(), r.trace.decode(), r.chim.decode()) if rc == 0 else (rc, "", "", ""))
            ob.lib().ocns_free(C.byref(r))
        return self._out(res)

    def mask(self, seqs, quals, hcr_mask, min_sr_length):
        masked, _, (bpt, bpn) = SO.mask_reads(seqs, quals, SO.mask_params_from_cfg(hcr_mask, min_sr_length))
        return masked, bpt, bpn
