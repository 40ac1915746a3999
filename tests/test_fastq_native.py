"""The short-read input's native 4-line FASTQ scan (pr_fastq4_scan / pr_fastq4_fill, correct.ShortReads)
against a numpy restatement of the same records, and the inputs it must hand to the general
record parser (FASTA, multi-line, CR line ends, mismatched quality lengths)."""
import numpy as np

from proovread_amd import correct


def _numpy_records(data: bytes):
    arr = np.frombuffer(data, np.uint8)
    nl = np.flatnonzero(arr == 10)
    starts = np.concatenate([[0], nl[3::4][:-1] + 1]).astype(np.int64)
    s0, s1 = (nl[0::4] + 1).astype(np.int64), nl[1::4].astype(np.int64)
    off = np.zeros(len(s0) + 1, np.int64)
    np.cumsum(s1 - s0, out=off[1:])
    pool = np.concatenate([correct.NT4[arr[a:b]] for a, b in zip(s0, s1)]) if len(s0) else np.zeros(0, np.uint8)
    return starts, off, pool


def test_native_fastq_matches_numpy_records():
    rng = np.random.default_rng(7)
    recs = []
    for i in range(500):
        n = int(rng.integers(0, 200))
        seq = rng.choice(np.frombuffer(b"ACGTNacgtnRY", np.uint8), n).tobytes()
        recs.append(b"@r%d extra words\n%s\n+%s\n%s\n" % (i, seq, b"" if i % 2 else b"r%d" % i, b"I" * n))
    data = b"".join(recs)
    got = correct._fastq4_native(data)
    want = _numpy_records(data)
    assert got is not None
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    sr = correct.ShortReads(data, chunk_number=10)
    assert np.array_equal(sr.pool, want[2]) and np.array_equal(sr.off, want[1])


def test_native_fastq_rejects_other_layouts():
    for bad in (b"", b">a\nACGT\n", b"@a\nACGT\n+\nIII\n", b"@a\r\nACGT\n+\nIIII\n", b"@a\nACGT\n+\nIIII",
                b"@a\nACGT\n-\nIIII\n", b"@a\nAC\nGT\n+\nIIII\n"):
        assert correct._fastq4_native(bad) is None, bad
    # the general parser still reads FASTA
    sr = correct.ShortReads(b">a\nACGT\nAC\n>b\nGG\n")
    assert sr.off.tolist() == [0, 6, 8]
