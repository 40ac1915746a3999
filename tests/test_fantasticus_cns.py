"""Consensus parity on the reference's bundled sample: 11 long reads of
sample/F.antasticus_long_error.fq (IUPAC codes included) with alignments of short reads
simulated from the sample genome (seeded by the product front end, extended by the SW
oracle), expected outputs from the reference Perl engine
(tests/golden/fantasticus/cns_expected.txt, regen_fantasticus.sh).

CPU: the C oracle reproduces the Perl outputs byte-exactly.  GPU: libprgpu's consensus
does too (single reads and one batched launch per parameter set)."""
from pathlib import Path

import pytest

import casefmt
import oracle_bind
from cns_case_util import case_inputs, params_key

GOLD = Path(__file__).resolve().parent / "golden" / "fantasticus"
CASES = casefmt.read_cases(GOLD / "cns_cases.txt")
EXPECT = casefmt.read_expect(GOLD / "cns_expected.txt")


def test_fixture_shape():
    assert len(CASES) == 11 and sum(len(c.sam) for c in CASES) > 1000
    assert any(any(ch not in "ACGTacgt" for ch in c.ref[1]) for c in CASES)   # IUPAC reference bases
    assert not any(EXPECT[c.name].error for c in CASES)


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_oracle_matches_reference_on_sample(case):
    e = EXPECT[case.name]
    r = oracle_bind.run_case(case)
    assert r["rc"] == 0
    assert r["fastq"].rstrip("\n").split("\n") == e.fastq
    assert r["trace"] == e.trace
    assert [l for l in r["chim"].split("\n") if l] == e.chim
    assert r["kept"] == e.kept


def _check(case, r):
    e = EXPECT[case.name]
    assert r.status == 0, (case.name, r.status)
    assert r.fastq.rstrip("\n").split("\n") == e.fastq, case.name
    assert r.trace == e.trace, case.name
    assert r.chim_lines() == e.chim, case.name
    assert "".join(str(int(x)) for x in r.kept) == e.kept, case.name


@pytest.mark.gpu
def test_gpu_matches_reference_on_sample():
    from proovread_amd import cns
    groups = {}
    for c in CASES:
        lr, alns, params = case_inputs(c)
        _check(c, cns.run_chunk([lr], [alns], params)[0])
        groups.setdefault(params_key(params), (params, []))[1].append((c, lr, alns))
    for params, items in groups.values():
        res = cns.run_chunk([x[1] for x in items], [x[2] for x in items], params)
        for (c, _, _), r in zip(items, res):
            _check(c, r)
