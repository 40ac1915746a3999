"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

Pure-Python restatement of proovread's read post-processing (SURVEY.md §8f.2,
§8f.4), for small inputs:

  qual_lcs      Fastq::Seq::qual_lcs (lib/Fastq/Seq.pm:709-717) with the range /
                min-length setters (Seq.pm:226-228, 322-367): maximal runs of
                quality chars inside [phred_min, phred_max], length >= min.
  mask_hcrs     the high-confidence-region masking that `SeqFilter --phred-mask`
                applies per iteration (bin/proovread:1701-1716).  SeqFilter is an
                absent submodule (.gitmodules:1-3); the algorithm is restated from
                its in-tree predecessor, sam2cns:806-951 (`mask_hcrs`, commented
                out there with "DEPRECATED, using SeqFilter now") and its
                parameter setup sam2cns:416-434, with the hcr-mask fields
                (proovread.cfg:230-242) mapped as
                  phred-min,phred-max -> Qual_lcs_range
                  mask-min-len        -> hcr_min_length
                  unmask-min-len      -> lcr_min_length
                  mask-reduce         -> hcr_sticky_length (per side)
                  mask-end-ratio      -> lcr_end_ratio
                  Qual_lcs_min_length = hcr_min + 2 * sticky (sam2cns:434).
                Pinning: the HCR search (qual_lcs) is checked against the
                reference module's own output (tests/golden/seqfilter_expected.txt,
                gen_seqfilter_golden.pl).  The sticky / end / gap rounds are
                restated from reading the commented-out sub, which cannot be run
                without extracting its text (not done); they and the
                field mapping onto SeqFilter are parity unpinned.
  qual_window   Fastq::Seq::qual_window and its _qw_slide_* helpers (Seq.pm:
                1064-1160), the windows `SeqFilter --trim-win mean,min` keeps
                (proovread.cfg:152-155), including the Perl quirks (low-slide
                window update subtracts X[I-W+1]; `A || B && return` precedence).
"""
from __future__ import annotations

import copy
import dataclasses
from typing import List, Sequence, Tuple


# ---------------------------------------------------------------- masking

@dataclasses.dataclass
class MaskParams:
    phred_min: int = 20
    phred_max: int = 41
    mask_min_len: int = 80
    unmask_min_len: int = 130
    mask_reduce: int = 60
    end_ratio: float = 0.7
    phred_offset: int = 33


def mask_params_from_cfg(hcr_mask: str, min_sr_length: int) -> MaskParams:
    """proovread:1702-1705: fields 2 and 3 scale with the short-read length (given for 100 bp)."""
    f = hcr_mask.split(",")
    m2 = int(float(f[2]) * min_sr_length / 100 + .5)
    m3 = int(float(f[3]) * min_sr_length / 100 + .5)
    return MaskParams(int(f[0]), int(f[1]), m2, m3, int(f[4]), float(f[5]))


def qual_lcs(qual: bytes, lo_char: int, hi_char: int, min_len: int) -> List[List[int]]:
    """Maximal runs of chars in [lo_char, hi_char] of length >= min_len, in order (Seq.pm:709-717)."""
    out = []
    n = len(qual)
    i = 0
    while i < n:
        if lo_char <= qual[i] <= hi_char:
            j = i
            while j < n and lo_char <= qual[j] <= hi_char:
                j += 1
            if j - i >= max(min_len, 1):
                out.append([i, j - i])
            i = j
        else:
            i += 1
    return out


def mask_hcrs(qual: bytes, P: MaskParams) -> Tuple[List[List[int]], List[List[int]]]:
    """-> (HCRs as found, MCRs actually masked), each [offset, length] (sam2cns:807-946)."""
    sticky, hcr_min, lcr_min = P.mask_reduce, P.mask_min_len, P.unmask_min_len
    L = len(qual)
    hcrs = qual_lcs(qual, P.phred_min + P.phred_offset, P.phred_max + P.phred_offset, hcr_min + 2 * sticky)
    if not hcrs:
        return [], []
    found = copy.deepcopy(hcrs)
    for h in hcrs:   # sticky ends
        h[0] += sticky
        h[1] -= 2 * sticky
    # head: unmask to lcr_min or mask the start completely
    short = lcr_min - hcrs[0][0]
    if short > 0:
        if short < P.end_ratio * lcr_min:
            hcrs[0][1] -= short
            if hcrs[0][1] < hcr_min:
                hcrs.pop(0)
            else:
                hcrs[0][0] += short
        else:
            hcrs[0][1] += hcrs[0][0]
            hcrs[0][0] = 0
    # tail
    if hcrs:
        short = lcr_min - (L - (hcrs[-1][0] + hcrs[-1][1]))
        if short > 0:
            if short < P.end_ratio * lcr_min:
                hcrs[-1][1] -= short
                if hcrs[-1][1] < hcr_min:
                    hcrs.pop()
            else:
                hcrs[-1][1] += lcr_min - short
    # gaps shorter than lcr_min: shrink both neighbours; drop HCRs that become too short
    while hcrs:
        tmp = copy.deepcopy(hcrs)
        shorts = []
        i = 0
        while i < len(hcrs) - 1:
            ha, hb = tmp[i], tmp[i + 1]
            s = lcr_min - (hb[0] - (ha[0] + ha[1]))
            if s > 0:
                a = s // 2
                b = a + s % 2
                ha[1] -= a
                if ha[1] < hcr_min:
                    shorts.append(i)
                hb[0] += b
                hb[1] -= b
            i += 1
        if tmp[i][1] < hcr_min:
            shorts.append(i)
        clean: List[int] = []
        for x in shorts:
            if clean and x - 1 == clean[-1]:
                # sam2cns:914 compares a length with an array reference (its address):
                # always true, so the later of two adjacent short HCRs replaces the earlier
                clean.pop()
            clean.append(x)
        if not clean:
            hcrs = tmp
            break
        for k, x in enumerate(clean):
            del hcrs[x - k]
    return found, hcrs


def mask_seq(seq: bytes, mcrs: Sequence[Sequence[int]]) -> bytes:
    s = bytearray(seq)
    for o, l in mcrs:
        if l > 0:
            s[o:o + l] = b"N" * l
    return bytes(s)


def mask_reads(seqs: Sequence[bytes], quals: Sequence[bytes], P: MaskParams):
    """-> masked sequences, MCR lists, (bpt, bpN) as `--base-content N` counts them."""
    out, mcrs = [], []
    bpt = bpn = 0
    for s, q in zip(seqs, quals):
        _, m = mask_hcrs(q, P)
        ms = mask_seq(s, m)
        out.append(ms)
        mcrs.append(m)
        bpt += len(ms)
        bpn += ms.count(b"N")
    return out, mcrs, (bpt, bpn)


# ---------------------------------------------------------------- trim windows

@dataclasses.dataclass
class WinParams:
    size: int = 10          # Qual_window_size
    soft: int = 25          # Qual_window_min_score_soft (mean)
    hard: int = 3           # Qual_window_min_score_hard (absolute)
    min_len: int = 10       # Qual_window_min_strecht_length

    @classmethod
    def trim_win(cls, spec: str):
        """`--trim-win mean,min` (proovread.cfg:153 "12,5")."""
        a, b = spec.split(",")
        return cls(soft=int(a), hard=int(b))


def qual_window(phreds: Sequence[int], P: WinParams) -> List[Tuple[int, int]]:
    """Fastq::Seq::qual_window (Seq.pm:1064-1160): [(offset, length)] in order."""
    X = list(phreds)
    n = len(X)
    W, S, H = P.size, P.soft, P.hard
    SW = S * W
    st = {"I": -1, "WX": 0}

    def init():
        if not (st["I"] + W < n):
            return False
        st["WX"] = 0
        for _ in range(W):
            st["I"] += 1
            if X[st["I"]] < H:
                return False
            st["WX"] += X[st["I"]]
        return True

    def low():
        I = st["I"]
        if X[I] < H:
            return False
        if not (st["WX"] < SW) and X[I - W + 1] > S:
            return True
        while True:
            I += 1
            if I >= n:
                break
            st["I"] = I
            if X[I] < H:
                return False
            st["WX"] += X[I] - X[I - W + 1]
            if not (st["WX"] < SW) and X[I - W + 1] > S:
                return True
        st["I"] = n - 1
        return False

    def high():
        o = st["I"] - W + 1
        I = st["I"]
        while True:
            I += 1
            if I >= n:
                break
            st["WX"] += X[I] - X[I - W]
            if st["WX"] < SW or X[I] < H:
                break
        I -= 1
        st["I"] = I
        j = I
        while X[j] < S:
            j -= 1
        l = j - o + 1
        return (o, l) if l >= P.min_len else None

    out = []
    while st["I"] < n - W:
        if not init():
            continue
        if not low():
            continue
        h = high()
        if h:
            out.append(h)
    return out
