"""Pin the consensus oracle (oracle/cns_oracle.c) to the reference.

The golden vectors in tests/golden/cns_expected.txt were produced by running
the reference Perl engine (lib/Sam/Seq.pm via tests/golden/gen_cns_golden.pl)
on tests/golden/cns_cases.txt.  Parity bar: byte-exact FASTQ, trace, chimera
lines and kept-alignment flags; error cases must error.
"""
from pathlib import Path

import pytest

import casefmt
import oracle_bind

GOLD = Path(__file__).resolve().parent / "golden"
CASES = casefmt.read_cases(GOLD / "cns_cases.txt")
EXPECT = casefmt.read_expect(GOLD / "cns_expected.txt")


def test_phred_tables_match_reference_values():
    L = oracle_bind.lib()
    # Seq.pm:151-156 probed values (perl -MSam::Seq: Phreds2freqs(3,20,30,40))
    assert [L.ocns_phred2freq(p) for p in (3, 20, 30, 40)] == [0.08, 3.33, 7.5, 13.33]
    assert L.ocns_freq2phred(0.0) == 0
    assert L.ocns_freq2phred(13.33) == 40
    assert L.ocns_freq2phred(1000.0) == 40


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_oracle_matches_reference(case):
    e = EXPECT[case.name]
    r = oracle_bind.run_case(case)
    if e.error:
        assert r["rc"] != 0
        return
    assert r["rc"] == 0
    assert r["fastq"].rstrip("\n").split("\n") == e.fastq
    assert r["trace"] == e.trace
    got_chim = [l for l in r["chim"].split("\n") if l]
    assert got_chim == e.chim
    assert r["kept"] == e.kept
