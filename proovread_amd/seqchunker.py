"""`SeqChunker` drop-in for proovread's short-read sampling.

proovread samples each iteration's short reads with
    SeqChunker --chunk-number 1000 --chunk-step 20 --chunks-per-step K --first-chunk F FILES | bwa mem ...
(cov2seqchunker, bin/proovread:2085-2102; run_bwa :1293-1299).  SeqChunker is an
absent submodule (.gitmodules:7-9); this restates its sampling as documented by
its options (parity unpinned):

  * the input files are taken as one byte stream; with --chunk-number N the
    stream is cut into N chunks of ceil(bytes / N) bytes (--chunk-size S: chunks
    of S bytes, k/M/G suffixes), and every record belongs to the chunk its first
    byte falls into (a chunk boundary moves to the next record start);
  * chunks are numbered from 1; the chunks written are F, F+1, ..., F+K-1, then
    the same K chunks of every following step of --chunk-step chunks, up to
    --last-chunk (default: the last);
  * records are written unchanged, to stdout or, with --out PATTERN containing
    a printf integer (e.g. pb-%03d.fq), one file per chunk.
"""
from __future__ import annotations

import argparse
import math
import re
import sys
from typing import Iterator, List, Optional, Tuple


def _size(s: str) -> int:
    m = re.fullmatch(r"\s*(\d+)\s*([kKmMgG]?)[bB]?\s*", s)
    if not m:
        raise ValueError(f"bad chunk size {s!r}")
    return int(m.group(1)) * {"": 1, "k": 1 << 10, "m": 1 << 20, "g": 1 << 30}[m.group(2).lower()]


def records(data: bytes) -> Iterator[Tuple[int, int]]:
    """(start, end) byte ranges of the FASTA / FASTQ records of data."""
    n = len(data)
    i = 0
    while i < n and data[i] in b"\r\n":
        i += 1
    if i >= n:
        return
    fasta = data[i:i + 1] == b">"
    if not fasta and data[i:i + 1] != b"@":
        raise ValueError("input is neither FASTA nor FASTQ")
    if fasta:
        while i < n:
            j = data.find(b"\n>", i)
            end = n if j < 0 else j + 1
            yield i, end
            i = end
        return
    while i < n:
        if data[i] in b"\r\n":
            i += 1
            continue
        p = i
        for _ in range(4):
            j = data.find(b"\n", p)
            p = n if j < 0 else j + 1
        yield i, p
        i = p


def select(n_chunks: int, first: int, step: int, per_step: int, last: Optional[int] = None) -> List[int]:
    last = n_chunks if last is None else min(last, n_chunks)
    if step <= 0:
        step, per_step = n_chunks, n_chunks
    return [k for k in range(max(first, 1), last + 1) if (k - first) % step < per_step]


def chunk(data: bytes, n_chunks: int = 0, chunk_size: int = 0) -> Tuple[int, List[List[Tuple[int, int]]]]:
    total = len(data)
    if chunk_size <= 0:
        n_chunks = max(1, n_chunks)
        chunk_size = max(1, math.ceil(total / n_chunks)) if total else 1
    else:
        n_chunks = max(1, math.ceil(total / chunk_size))
    out: List[List[Tuple[int, int]]] = [[] for _ in range(n_chunks)]
    for s, e in records(data):
        out[min(s // chunk_size, n_chunks - 1)].append((s, e))
    return n_chunks, out


def main(argv: Optional[List[str]] = None, stdout=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    stdout = stdout or sys.stdout.buffer
    ap = argparse.ArgumentParser(prog="SeqChunker")
    ap.add_argument("files", nargs="*")
    ap.add_argument("-n", "--chunk-number", type=int, default=0)
    ap.add_argument("-s", "--chunk-size", default=None)
    ap.add_argument("-x", "--chunk-step", type=int, default=0)
    ap.add_argument("-y", "--chunks-per-step", type=int, default=1)
    ap.add_argument("-f", "--first-chunk", type=int, default=1)
    ap.add_argument("-l", "--last-chunk", type=int, default=None)
    ap.add_argument("-o", "--out", default=None)
    ap.add_argument("-q", "--quiet", action="store_true")
    a = ap.parse_args(argv)
    data = b"".join(open(f, "rb").read() for f in a.files) if a.files else sys.stdin.buffer.read()
    size = _size(a.chunk_size) if a.chunk_size else 0
    if not size and a.chunk_number <= 0:
        print("SeqChunker: --chunk-number or --chunk-size required", file=sys.stderr)
        return 1
    n, chunks = chunk(data, a.chunk_number, size)
    for k in select(n, a.first_chunk, a.chunk_step, a.chunks_per_step, a.last_chunk):
        blob = b"".join(data[s:e] for s, e in chunks[k - 1])
        if a.out:
            with open(a.out % k, "wb") as fh:
                fh.write(blob)
        else:
            stdout.write(blob)
    if hasattr(stdout, "flush"):
        stdout.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
