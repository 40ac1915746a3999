"""Consensus parity at full size against the reference Perl engine (tests/golden/scale/,
make_scale_cases.py + regen_scale.sh): 30 long reads of ~10 kb each, in two task settings --

  bwa-sr-1       raw 15 %-error reads, ~940 alignments per read, cap 11.25, --use-ref-qual
  bwa-sr-finish  the reads corrected by that iteration, ~1,800 alignments per read (30x,
                 finish options, -D .75), cap 22.5, --no-use-ref-qual, --detect-chimera, six
                 chimeric reads (bin/proovread:1572-1579; lib/Sam/Seq.pm:774-889;
                 bin/bam2cns:461-491)

The expected FASTQ, trace, chimera lines and kept flags are the Perl engine's own outputs.
CPU: the C oracle reproduces them byte for byte.  GPU: libprgpu's consensus does too, one
batched launch per setting (the way pr_cns_run is called per bam2cns chunk)."""
from pathlib import Path

import pytest

import casefmt
import oracle_bind
from cns_case_util import case_inputs

GOLD = Path(__file__).resolve().parent / "golden" / "scale"
SETS = ("bwa_sr1", "finish")


def _load(k):
    return (casefmt.read_cases(GOLD / f"{k}_cases.txt.gz"), casefmt.read_expect(GOLD / f"{k}_expected.txt.gz"))


_CACHE = {}


def load(k):
    if k not in _CACHE:
        _CACHE[k] = _load(k)
    return _CACHE[k]


@pytest.mark.parametrize("k", SETS)
def test_fixture_shape(k):
    cases, expect = load(k)
    assert len(cases) >= 30
    assert all(len(c.ref[1]) >= 8000 for c in cases)
    assert sum(len(c.sam) for c in cases) >= 30 * (900 if k == "bwa_sr1" else 1500)
    assert not any(expect[c.name].error for c in cases)
    if k == "finish":
        assert all(c.p("detect_chimera") == "1" and c.p("use_ref_qual") == "0" for c in cases)
        assert sum(len(expect[c.name].chim) for c in cases) > 100


def _check(case, e, fastq, trace, chim, kept):
    assert fastq == e.fastq, case.name
    assert trace == e.trace, case.name
    assert chim == e.chim, case.name
    assert kept == e.kept, case.name


@pytest.mark.parametrize("k", SETS)
def test_oracle_matches_reference_at_scale(k):
    cases, expect = load(k)
    for c in cases:
        r = oracle_bind.run_case(c)
        assert r["rc"] == 0, c.name
        _check(c, expect[c.name], r["fastq"].rstrip("\n").split("\n"), r["trace"],
               [ln for ln in r["chim"].split("\n") if ln], r["kept"])


@pytest.mark.gpu
@pytest.mark.parametrize("k", SETS)
def test_gpu_matches_reference_at_scale(k):
    from proovread_amd import cns
    cases, expect = load(k)
    items = [case_inputs(c) for c in cases]
    params = items[0][2]
    res = cns.run_chunk([x[0] for x in items], [x[1] for x in items], params)
    for c, r in zip(cases, res):
        assert r.status == 0, (c.name, r.status)
        _check(c, expect[c.name], r.fastq.rstrip("\n").split("\n"), r.trace, r.chim_lines(),
               "".join(str(int(x)) for x in r.kept))
