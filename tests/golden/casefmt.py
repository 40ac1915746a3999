"""Text format shared by the consensus golden fixtures, the C oracle tests and
the GPU parity tests.

A case file holds one or more cases::

    >>CASE name
    >>PARAM coverage 11.25
    >>PARAM use_ref_qual 1
    ...
    >>REF
    @id [desc with MCRn:off,len tags]
    SEQ
    +
    QUAL
    >>SAM
    <SAM lines of alignments against that long read, in BAM (coordinate) order>
    >>END

An expected-output file holds, per case::

    >>CASE name
    >>ERROR 1                      (only if the reference died)
    >>FASTQ
    @id\nSEQ\n+\nQUAL
    >>TRACE
    MMMDI...
    >>CHIM
    id\tfrom\tto\tscore   (zero or more lines)
    >>KEPT
    0110...
    >>END
"""
from __future__ import annotations

import dataclasses
import gzip
from typing import Dict, List


def _open(path):
    return gzip.open(path, "rt") if str(path).endswith(".gz") else open(path)

DEFAULT_PARAMS = {
    "coverage": "11.25",
    "use_ref_qual": "1",
    "detect_chimera": "0",
    "max_ins_length": "0",
    "qual_weighted": "0",
    "noref": "0",
}


@dataclasses.dataclass
class Case:
    name: str
    params: Dict[str, str]
    ref: List[str]          # 4 FASTQ lines (without newline)
    sam: List[str]          # SAM lines (without newline)

    @property
    def ref_id(self) -> str:
        return self.ref[0][1:].split()[0]

    @property
    def ref_desc(self) -> str:
        parts = self.ref[0][1:].split(None, 1)
        return parts[1] if len(parts) > 1 else ""

    def p(self, k):
        return self.params.get(k, DEFAULT_PARAMS[k])


@dataclasses.dataclass
class Expect:
    name: str
    error: bool
    fastq: List[str]
    trace: str
    chim: List[str]
    kept: str


def write_cases(path, cases: List[Case]):
    with open(path, "w") as fh:
        for c in cases:
            fh.write(f">>CASE {c.name}\n")
            for k, v in c.params.items():
                fh.write(f">>PARAM {k} {v}\n")
            fh.write(">>REF\n")
            for l in c.ref:
                fh.write(l + "\n")
            fh.write(">>SAM\n")
            for l in c.sam:
                fh.write(l + "\n")
            fh.write(">>END\n")


def read_cases(path) -> List[Case]:
    out = []
    cur = None
    sect = None
    with _open(path) as fh:
        for line in fh:
            line = line.rstrip("\n")
            if line.startswith(">>CASE "):
                cur = Case(line[7:], {}, [], [])
                sect = None
            elif line.startswith(">>PARAM "):
                _, k, v = line.split(" ", 2)
                cur.params[k] = v
            elif line == ">>REF":
                sect = "ref"
            elif line == ">>SAM":
                sect = "sam"
            elif line == ">>END":
                out.append(cur)
                cur = None
            elif sect == "ref":
                cur.ref.append(line)
            elif sect == "sam":
                if line:
                    cur.sam.append(line)
    return out


def read_expect(path) -> Dict[str, Expect]:
    out = {}
    cur = None
    sect = None
    with _open(path) as fh:
        for line in fh:
            line = line.rstrip("\n")
            if line.startswith(">>CASE "):
                cur = Expect(line[7:], False, [], "", [], "")
                sect = None
            elif line.startswith(">>ERROR"):
                cur.error = True
            elif line in (">>FASTQ", ">>TRACE", ">>CHIM", ">>KEPT"):
                sect = line[2:].lower()
            elif line == ">>END":
                out[cur.name] = cur
                cur = None
            elif sect == "fastq":
                cur.fastq.append(line)
            elif sect == "trace":
                cur.trace += line
            elif sect == "chim":
                if line:
                    cur.chim.append(line)
            elif sect == "kept":
                cur.kept += line
    return out
