"""Final trimming windows: libprgpu.so's host pr_trim_windows against
the reference's own Fastq::Seq::qual_window outputs (tests/golden/seqfilter_expected.txt,
WIN cases, made by gen_seqfilter_golden.pl) and against the oracle restatement on
random quality strings.  Host code: no GPU needed."""
import random
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import seqfilter_oracle as O  # noqa: E402

GOLD = ROOT / "tests" / "golden"


def _win_cases():
    cases = (GOLD / "seqfilter_cases.txt").read_text().splitlines()
    exp = (GOLD / "seqfilter_expected.txt").read_text().splitlines()
    for c, e in zip(cases, exp):
        if c.startswith("WIN"):
            f = c.split("\t")
            want = [tuple(int(x) for x in p.split(",")) for p in e.split("\t", 1)[1].split()]
            yield tuple(map(int, f[1:5])), f[5].encode(), want


def _p(size, soft, hard, minl):
    from proovread_amd import trim
    p = trim.params()
    p.size, p.soft, p.hard, p.min_len = size, soft, hard, minl
    return p


def test_trim_windows_match_reference_goldens():
    from proovread_amd import trim
    n = nw = 0
    for prm, q, want in _win_cases():
        assert O.qual_window([c - 33 for c in q], O.WinParams(*prm)) == want
        assert trim.windows([q], _p(*prm))[0] == want, (prm, len(q))
        n += 1
        nw += len(want)
    assert n == 80 and nw > 100


@pytest.mark.parametrize("seed", [1, 2])
def test_trim_windows_batch_matches_oracle(seed):
    from proovread_amd import trim
    rng = random.Random(seed)
    for _ in range(5):
        prm = (rng.choice([3, 5, 10, 20]), rng.randint(5, 30), rng.randint(0, 12), rng.randint(1, 40))
        quals = []
        for _ in range(rng.randint(0, 200)):
            L = rng.choice([0, 1, 9, 10, 11, 100, 1000, 4000])
            ph, hi = [], rng.random() < 0.5
            while len(ph) < L:
                k = rng.randint(1, rng.choice([5, 40, 400]))
                ph += [rng.randint(15, 41) if hi else rng.randint(0, 20) for _ in range(k)]
                hi = not hi
            quals.append(bytes(33 + x for x in ph[:L]))
        got = trim.windows(quals, _p(*prm), threads=rng.choice([1, 3, 0]))
        assert got == [O.qual_window([c - 33 for c in q], O.WinParams(*prm)) for q in quals]


def test_trim_params_parse():
    from proovread_amd import trim
    p = trim.params("12,5")
    assert (p.size, p.soft, p.hard, p.min_len) == (10, 12, 5, 10)
    with pytest.raises(RuntimeError):
        trim.params("12")
