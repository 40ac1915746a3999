"""Minimal BAM writer for tests (SAM v1 spec §4: BGZF blocks + binary records).

Used to feed the bam2cns drop-in the same alignments a golden case holds as SAM
text, without samtools.  Writes real BGZF (BC extra field, EOF marker) so the
files are readable by samtools as well.
"""
from __future__ import annotations

import struct
import zlib
from typing import Dict, List, Sequence, Tuple

_NT16 = {c: i for i, c in enumerate("=ACMGRSVTWYHKDBN")}
_OPS = "MIDNSHP=X"
_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _bgzf_block(data: bytes) -> bytes:
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    comp = c.compress(data) + c.flush()
    bsize = len(comp) + 25
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
    return hdr + comp + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def _reg2bin(beg: int, end: int) -> int:
    end -= 1
    for shift, off in ((14, 4681), (17, 585), (20, 73), (23, 9), (26, 1)):
        if beg >> shift == end >> shift:
            return off + (beg >> shift)
    return 0


def _cigar_ops(cig: str) -> List[int]:
    if cig == "*":
        return []
    out, num = [], ""
    for ch in cig:
        if ch.isdigit():
            num += ch
        else:
            out.append((int(num) << 4) | _OPS.index(ch))
            num = ""
    return out


def _aux(tags: Sequence[str]) -> bytes:
    out = b""
    for t in tags:
        tag, typ, val = t.split(":", 2)
        if typ == "i":
            out += tag.encode() + b"i" + struct.pack("<i", int(val))
        elif typ == "f":
            out += tag.encode() + b"f" + struct.pack("<f", float(val))
        elif typ == "A":
            out += tag.encode() + b"A" + val.encode()
        else:
            out += tag.encode() + b"Z" + val.encode() + b"\0"
    return out


def sam_line_to_record(line: str, ref_index: Dict[str, int]) -> bytes:
    f = line.rstrip("\n").split("\t")
    qname, flag, rname, pos, mapq, cig = f[0], int(f[1]), f[2], int(f[3]), int(f[4]), f[5]
    seq, qual = f[9], f[10]
    ops = _cigar_ops(cig)
    ref_len = sum(o >> 4 for o in ops if (o & 15) in (0, 2, 3, 7, 8)) or 1
    l_seq = 0 if seq == "*" else len(seq)
    sb = bytearray((l_seq + 1) // 2)
    for i in range(l_seq):
        sb[i >> 1] |= _NT16.get(seq[i].upper(), 15) << (4 * (1 - (i & 1)))
    qb = bytes([0xFF] * l_seq) if qual == "*" else bytes(ord(c) - 33 for c in qual[:l_seq])
    rn = qname.encode() + b"\0"
    rid = ref_index.get(rname, -1)
    body = struct.pack("<iiBBHHHiiii", rid, pos - 1, len(rn), mapq, _reg2bin(pos - 1, pos - 1 + ref_len),
                       len(ops), flag, l_seq, -1, -1, 0)
    body += rn + struct.pack(f"<{len(ops)}I", *ops) + bytes(sb) + qb + _aux(f[11:])
    return struct.pack("<i", len(body)) + body


def write_bam(path: str, refs: Sequence[Tuple[str, int]], sam_lines: Sequence[str]) -> None:
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join(f"@SQ\tSN:{n}\tLN:{l}\n" for n, l in refs)
    raw = b"BAM\x01" + struct.pack("<i", len(text)) + text.encode() + struct.pack("<i", len(refs))
    for n, l in refs:
        raw += struct.pack("<i", len(n) + 1) + n.encode() + b"\0" + struct.pack("<i", l)
    idx = {n: i for i, (n, _) in enumerate(refs)}
    raw += b"".join(sam_line_to_record(l, idx) for l in sam_lines)
    with open(path, "wb") as fh:
        for o in range(0, len(raw), 0xFF00):
            fh.write(_bgzf_block(raw[o:o + 0xFF00]))
        fh.write(_EOF)
