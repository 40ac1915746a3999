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


def test_gpu_scatter_fallback_path_matches_reference(monkeypatch):
    """The in-kernel scatter path (taken when a read's expanded pileup exceeds the
    per-workgroup scratch) forced for every read: same bytes as the reference."""
    from proovread_amd import cns
    monkeypatch.setenv("PRGPU_CNS_SCATTER", "1")
    n = 0
    for c in CASES:
        lr, alns, params = case_inputs(c)
        if params.qual_weighted:
            continue
        _check(c, cns.run_chunk([lr], [alns], params)[0])
        n += 1
    assert n > 50
