"""CPU stages for proovread_amd.correct's loop (TEST INFRASTRUCTURE ONLY).

Same interface as correct.GpuStages, computed by the oracles: the SW oracle ->
SAM order -> consensus oracle chain (oracle/cpu_chain.py) for an iteration, and
the mask_hcrs restatement (oracle/seqfilter_oracle.py) for SeqFilter
--phred-mask.  The GPU loop must reproduce this loop byte-for-byte.  The
exact-parity multi-rank layout (owned_iteration) is restated on the host: host
seeding of the rank's short-read shard, the bwa-mode oracle, SAM records sent to
the long reads' owners with the communicator's all-to-all (gloo in the CPU
tests), the -b/-l filter and samtools order, the consensus oracle."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import cpu_chain  # noqa: E402
import seqfilter_oracle as SO  # noqa: E402


class OracleStages:
    def __init__(self, workers: int = 4):
        self.workers = workers

    # -- the loop's stage interface (correct.GpuStages), the state held on the host
    def load(self, reads):
        self.ids, self.seqs, self.quals = list(reads.ids), list(reads.seqs), list(reads.quals)
        self.map = list(self.seqs)

    def task(self, task, sr, sr_off, params, bin_filter, comm=None, exact=False, mask_cfg=None, sr_ranges=None):
        from proovread_amd import correct, tasks as T
        finish = mask_cfg is None
        lr_map, lr_off = correct._pool(self.seqs if finish else self.map)   # finish: the unmasked reads
        lr_map = correct.NT4[lr_map]
        ref_seq, _ = correct._pool(self.seqs)
        ref_qual, _ = correct._pool(self.quals)
        mres = None
        if not exact:
            tk = correct._seed_tasks(lr_map, lr_off, sr, sr_off, T.options(task)[0], self.workers)
            n_tasks = int(len(tk))
            d = correct._seeds_dataset(lr_map, lr_off, sr, sr_off, tk)
            out = self.iteration(d, ref_seq, ref_qual, task, params, bin_filter=bin_filter)
            lo, hi = 0, len(self.ids)
        else:
            lo, hi, out, n_tasks, mres = self.owned_iteration(lr_map, lr_off, sr, sr_off, task, params, ref_seq,
                                                              ref_qual, bin_filter, comm, mask_cfg)
        seqs, quals, lines = [], [], []
        for rid, (st, s, q, ch) in zip(self.ids[lo:hi], out):
            if st != 0:
                raise RuntimeError(f"{task}: consensus of {rid} failed with status {st}")
            seqs.append(s)
            quals.append(q)
            lines += correct._rename(ch, rid)
        masked, bpt, bpn = [], 0, 0
        if mres is not None:
            masked, bpt, bpn = mres
        elif not finish and seqs:
            masked, bpt, bpn = self.mask(seqs, quals, mask_cfg[0], mask_cfg[1])
        if comm is not None and comm.world > 1:
            seqs, quals = comm.allgather_lists(seqs), comm.allgather_lists(quals)
            if not finish:
                masked = comm.allgather_lists(masked)
        self.seqs, self.quals = seqs, quals
        if not finish:
            self.map = masked
        return correct.TaskOut(n_tasks, lines if finish else [], bpt, bpn)

    def reads(self):
        from proovread_amd import correct
        return correct.LongReads(self.ids, self.seqs, self.quals)

    def masked(self):
        return list(self.map)

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

    def owned_iteration(self, lr_map, lr_off, sr, sr_off, task, params, ref_seq, ref_qual, bin_filter, comm,
                        mask_cfg=None):
        """correct.GpuStages.owned_iteration's contract on the host."""
        from proovread_amd import correct, exact_shard as ex, tasks as T
        world, rank = (comm.world, comm.rank) if comm is not None else (1, 0)
        s, e = ex.sr_range(len(sr_off) - 1, world, rank)
        tk = correct._seed_tasks(lr_map, lr_off, sr[sr_off[s]:sr_off[e]], np.asarray(sr_off[s:e + 1]) - sr_off[s],
                                 T.options(task)[0], 2)
        tk["sr"] += s
        d = correct._seeds_dataset(lr_map, lr_off, sr, sr_off, tk)
        recs = self.align(d, task)
        sams, lo, hi = records_by_owner(recs, sr, sr_off, lr_off, comm, bin_filter)
        ids = [f"lr{i}" for i in range(lo, hi)]
        seqs = [ref_seq[lr_off[i]:lr_off[i + 1]].tobytes() for i in range(lo, hi)]
        quals = [ref_qual[lr_off[i]:lr_off[i + 1]].tobytes() for i in range(lo, hi)]
        out = self.consensus(ids, seqs, quals, sams, params) if hi > lo else []
        mres = None
        if mask_cfg is not None:
            ok = [(x[1], x[2]) for x in out]
            mres = self.mask([x[0] for x in ok], [x[1] for x in ok], mask_cfg[0], mask_cfg[1]) if ok else ([], 0, 0)
        return lo, hi, out, int(len(tk)), mres


_ASC = np.frombuffer(b"ACGTN", np.uint8)


def records_by_owner(recs, sr, sr_off, lr_off, comm, bin_filter):
    """This rank's reported alignments (SAM order, read by read) go to the owners of their long
    reads (one all-to-all of fixed fields + one of CIGAR ops); the owner gets them
    source-rank-major, i.e. in the single run's read order, applies bwa-proovread's -b/-l
    filter in that order and returns, per owned long read, its SAM lines in samtools
    coordinate order (POS, strand, arrival)."""
    from proovread_amd import exact_shard as ex
    from proovread_amd.bwa_proovread import BinFilter, aln_length
    world, rank = (comm.world, comm.rank) if comm is not None else (1, 0)
    b = ex.lr_bounds(lr_off, world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    fix = np.array([r[:6] + (len(r[6]),) for r in recs], np.int32).reshape(-1, 7)
    own = np.searchsorted(b, fix[:, 1].astype(np.int64), side="right") - 1 if len(fix) else np.zeros(0, np.int64)
    order = np.argsort(own, kind="stable")
    counts = np.bincount(own, minlength=world).astype(np.int64)
    cig = [np.asarray(recs[i][6], np.int32) for i in order]
    cig_rows = np.concatenate(cig).reshape(-1, 1) if cig else np.zeros((0, 1), np.int32)
    per_dst = np.zeros(world, np.int64)
    for k, i in enumerate(order):
        per_dst[own[i]] += len(recs[i][6])
    if comm is None or world == 1:
        got, got_cig = fix[order], cig_rows.reshape(-1)
    else:
        got = comm.alltoallv_rows(np.ascontiguousarray(fix[order]), counts)
        got_cig = comm.alltoallv_rows(np.ascontiguousarray(cig_rows, np.int32), per_dst).reshape(-1)
    filt = BinFilter(*bin_filter) if bin_filter else None
    per_lr = [[] for _ in range(hi - lo)]
    c = 0
    for k in range(len(got)):
        srid, lr, strand, pos, score, flag, nc = (int(x) for x in got[k])
        ops = got_cig[c:c + nc]
        c += nc
        q = sr[sr_off[srid]:sr_off[srid + 1]]
        seq = (_ASC[np.where(q < 4, 3 - q, 4)][::-1] if strand else _ASC[q]).tobytes().decode()
        cg = "".join(f"{int(x) >> 4}{'MIDNSHP=X'[int(x) & 15]}" for x in ops)
        keep = filt.add(lr, pos + 1, aln_length(cg, len(q)), float(score)) if filt else None
        per_lr[lr - lo].append((pos, strand, k, keep, f"sr{srid}\t{flag}\tlr{lr}\t{pos + 1}\t60\t{cg}\t*\t0\t0\t"
                                                      f"{seq}\t*\tAS:i:{score}"))
    out = []
    for v in per_lr:
        if filt is not None:
            v = [x for x in v if filt.alive[x[3]]]
        out.append([x[4] for x in sorted(v, key=lambda x: (x[0], x[1], x[2]))])
    return out, lo, hi
