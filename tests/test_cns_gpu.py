"""GPU parity of the consensus stage (libprgpu.so, through the C-ABI) against
the reference golden vectors (tests/golden/cns_expected.txt, produced by the
Perl Sam::Seq engine) and against the C oracle on larger seeded inputs.

Bar: byte-exact FASTQ (sequence AND qualities), trace, chimera lines and
kept-alignment flags; cases where the reference dies must return an error.
"""
from pathlib import Path

import pytest

import casefmt
from cns_case_util import case_inputs, params_key

GOLD = Path(__file__).resolve().parent / "golden"
CASES = casefmt.read_cases(GOLD / "cns_cases.txt")
EXPECT = casefmt.read_expect(GOLD / "cns_expected.txt")

pytestmark = pytest.mark.gpu


def _check(case, r):
    e = EXPECT[case.name]
    if e.error:
        assert r.status != 0, case.name
        return
    assert r.status == 0, (case.name, r.status)
    assert r.fastq.rstrip("\n").split("\n") == e.fastq, case.name
    assert r.trace == e.trace, case.name
    assert r.chim_lines() == e.chim, case.name
    assert "".join(str(int(x)) for x in r.kept) == e.kept, case.name


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_gpu_matches_reference_single(case):
    from proovread_amd import cns
    lr, alns, params = case_inputs(case)
    if params.qual_weighted:
        with pytest.raises(RuntimeError, match="UNSUPPORTED"):
            cns.run_chunk([lr], [alns], params)
        return
    r = cns.run_chunk([lr], [alns], params)[0]
    _check(case, r)


def test_gpu_matches_reference_batched():
    """All cases sharing parameters in one launch (a bam2cns chunk)."""
    from proovread_amd import cns
    groups = {}
    for c in CASES:
        lr, alns, params = case_inputs(c)
        if params.qual_weighted or c.p("noref") == "1":
            continue
        groups.setdefault(params_key(params), (params, []))[1].append((c, lr, alns))
    n = 0
    for params, items in groups.values():
        res = cns.run_chunk([x[1] for x in items], [x[2] for x in items], params)
        for (c, _, _), r in zip(items, res):
            _check(c, r)
            n += 1
    assert n > 20


@pytest.mark.parametrize("batched", [False, True])
def test_gpu_large_geometry_matches_reference(monkeypatch, batched):
    """The large LDS geometry (state table 4096, 512-column windows: the rerun of reads
    whose tables outgrow the small one) forced for every read: same bytes as the
    reference, one read per launch and all reads of a parameter set in one launch."""
    from proovread_amd import cns
    monkeypatch.setenv("PRGPU_CNS_LARGE", "1")
    n = 0
    if not batched:
        for c in CASES:
            lr, alns, params = case_inputs(c)
            if params.qual_weighted:
                continue
            _check(c, cns.run_chunk([lr], [alns], params)[0])
            n += 1
        assert n > 50
        return
    groups = {}
    for c in CASES:
        lr, alns, params = case_inputs(c)
        if params.qual_weighted or c.p("noref") == "1":
            continue
        groups.setdefault(params_key(params), (params, []))[1].append((c, lr, alns))
    for params, items in groups.values():
        for (c, _, _), r in zip(items, cns.run_chunk([x[1] for x in items], [x[2] for x in items], params)):
            _check(c, r)
            n += 1
    assert n > 20


def _insertion_heavy_case(name, seed, L, n_aln, every, ins_len, coverage):
    """A long read whose alignments carry an insertion of ins_len random bases after every
    `every` reference bases: many distinct insertion states (ins_len 6) or many
    (column, state) pairs per window (ins_len 1, deep coverage)."""
    import random
    rng = random.Random(seed)
    ref = "".join(rng.choice("ACGT") for _ in range(L))
    starts = sorted(rng.randrange(0, L - 160) for _ in range(n_aln))
    sam = []
    for k, s in enumerate(starts):
        seq, cig, r = [], [], s
        while r < s + 150:
            m = min(every, s + 150 - r)
            seq.append(ref[r:r + m])
            cig.append(f"{m}M")
            r += m
            if r < s + 150:
                seq.append("".join(rng.choice("ACGT") for _ in range(ins_len)))
                cig.append(f"{ins_len}I")
        sq = "".join(seq)
        sam.append(f"sr{k}\t0\tlr\t{s + 1}\t60\t{''.join(cig)}\t*\t0\t0\t{sq}\t{'I' * len(sq)}\tAS:i:{300 + rng.randrange(200)}")
    return casefmt.Case(name, {"coverage": str(coverage)}, ["@lr", ref, "+", "$" * L], sam)


@pytest.mark.parametrize("kind", ["states", "pairs"])
def test_gpu_retry_geometry_matches_oracle(kind):
    """Reads that overflow the small geometry's tables (> 1024 distinct insertion states, or
    > 2048 (column, state) pairs in a 1024-column window) are rerun with the large one;
    the result equals the C oracle's."""
    import oracle_bind as ob
    from proovread_amd import cns
    c = (_insertion_heavy_case("many_states", 5, 3000, 150, 15, 6, 100.0) if kind == "states"
         else _insertion_heavy_case("many_pairs", 6, 2000, 1000, 10, 1, 400.0))
    lr, alns, params = case_inputs(c)
    r = cns.run_chunk([lr], [alns], params)[0]
    want = ob.run_case(c)
    assert want["rc"] == 0 and r.status == 0, (want["rc"], r.status)
    assert r.fastq == want["fastq"]
    assert r.trace == want["trace"]
