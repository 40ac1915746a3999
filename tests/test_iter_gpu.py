"""End-to-end parity of one GPU iteration (pr_iter_*: SW -> device hand-off ->
consensus) against the CPU chain SW oracle -> SAM -> coordinate sort ->
consensus oracle, on seeded synthetic long/short reads.  Bar: byte-exact
corrected reads (sequence and qualities), traces and chimera records.  The task
list is either the simulation truth or the product's own seeding front end
(pr_seed_map, bwa mem seeding + chaining restated), as bench.py uses it."""
import numpy as np
import pytest

import oracle_bind as ob
from pipeline_oracle import consensus_cases, sam_for_tasks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seeds", ["truth", "host", "truth-slot16", "host-binfilter", "bwa", "bwa-binfilter"])
@pytest.mark.parametrize("finish", [False, True])
def test_iteration_matches_cpu_chain(finish, seeds, monkeypatch):
    """truth-slot16: CIGAR slots forced to 16 ops, so most alignments reach the consensus
    through the overflow pass's spill area (the hand-off reads per-task CIGAR starts).
    host-binfilter: bwa-proovread's -b 20 -l 20*15 filter on the device before the hand-off
    (bin/proovread:1302-1313), against the oracle chain with the same filter; the coverage
    is raised so the filter drops alignments."""
    from proovread_amd import cns, iteration, seed, sw, synth
    if seeds.endswith("slot16"):
        monkeypatch.setenv("PRGPU_SW_CIG_SLOT", "16")
    binf = (20, 20.0 * 15) if seeds.endswith("binfilter") else None
    d = synth.simulate(31 + finish, 40000, 40, 2500, 40 if binf else 15, sr_frac=1.0)
    if seeds.startswith("host") or seeds.startswith("bwa"):
        ix = seed.SeedIndex(d.lr_seq, d.lr_off)
        tk = ix.map(d.sr_seq, d.sr_off, seed.default_opts(finish), threads=4)
        if seeds.startswith("host"):   # single-seed tasks: each chain's first seed
            tk = tk[tk["rank"] == 0]
        d = (synth.with_seeds if seeds.startswith("bwa") else synth.with_seeded_tasks)(d, tk)
        ix.close()
        assert len(d.t_sr) > 10 * d.n_lr
    task = "bwa-sr-finish" if finish else "bwa-sr"
    params = {"coverage": "22.5" if finish else "11.25", "use_ref_qual": "0" if finish else "1",
              "detect_chimera": "1" if finish else "0"}
    it = iteration.Iteration(d)
    cp = cns.CnsParams(coverage=float(params["coverage"]), use_ref_qual=params["use_ref_qual"] == "1",
                       detect_chimera=params["detect_chimera"] == "1")
    opts = sw.default_opts(finish=finish)
    if binf:
        opts.bin_size, opts.bin_length = binf
    it.launch(opts, cp)
    got = it.results()
    if seeds.startswith("bwa"):   # bwa mode: the oracle chain over every seed (aln_oracle.c)
        import sys
        from pathlib import Path
        sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
        import cpu_chain
        _, _, want, _ = cpu_chain.run_sample(d, range(d.n_lr), task=task, coverage=float(params["coverage"]),
                                             use_ref_qual=params["use_ref_qual"] == "1", workers=4,
                                             detect_chimera=params["detect_chimera"] == "1", full=True,
                                             bin_filter=binf)
        for i, (g, (rc, fq, trace, chim)) in enumerate(zip(got, want)):
            assert rc == 0 and g.status == 0, (i, rc, g.status)
            assert g.fastq == fq.replace(f"@lr{i}", f"@lr{i}"), i
            assert g.trace == trace, i
            assert "".join(l + "\n" for l in g.chim_lines()) == chim, i
        return
    sams = sam_for_tasks(d, task, bin_filter=binf)
    if binf:   # the filter must bite: fewer records than the unfiltered chain
        assert sum(map(len, sams.values())) < sum(map(len, sam_for_tasks(d, task).values()))
    cases = consensus_cases(d, sams, params)
    n_checked = 0
    for c, g in zip(cases, got):
        want = ob.run_case(c)
        assert want["rc"] == 0
        assert g.status == 0, (c.name, g.status)
        assert g.fastq == want["fastq"], c.name
        assert g.trace == want["trace"], c.name
        assert "".join(l + "\n" for l in g.chim_lines()) == want["chim"], c.name
        n_checked += 1
    assert n_checked == d.n_lr
