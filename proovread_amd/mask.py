"""Masking of corrected long reads on the GPU (pr_mask_* / pr_iter_mask of libprgpu.so).

proovread masks the high-confidence regions of every corrected read after an
iteration with `SeqFilter --phred-mask <hcr-mask> --base-content N --tsv -`
(bin/proovread:1701-1716; hcr-mask proovread.cfg:230-242, scaled to the
short-read length at proovread:1702-1705).  The masked reads are the next
iteration's mapping reference; bpN/bpt decides whether iterations are skipped
(mask_shortcut_frac, proovread:2026-2047).  Algorithm: csrc/mask_core.h.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _abi


class MaskParams(C.Structure):
    _fields_ = [("phred_min", C.c_int32), ("phred_max", C.c_int32), ("mask_min_len", C.c_int32),
                ("unmask_min_len", C.c_int32), ("mask_reduce", C.c_int32), ("end_ratio", C.c_double),
                ("phred_offset", C.c_int32)]


def _setup(L):
    if getattr(L, "_mask_ready", False):
        return
    L.pr_mask_params_default.argtypes = [C.POINTER(MaskParams)]
    L.pr_mask_params_parse.argtypes = [C.c_char_p, C.c_int32, C.POINTER(MaskParams)]
    L.pr_mask_bound.argtypes = [C.POINTER(MaskParams), C.c_int32, C.c_void_p, C.POINTER(C.c_int64)]
    L.pr_mask_run.argtypes = [C.c_void_p, C.POINTER(MaskParams), C.c_int32] + [C.c_void_p] * 8
    L.pr_iter_mask.argtypes = [C.c_void_p, C.POINTER(MaskParams), C.c_void_p]
    L.pr_iter_mask_download.argtypes = [C.c_void_p, C.c_void_p]
    L._mask_ready = True


def params(hcr_mask: Optional[str] = None, min_sr_length: int = 100, phred_offset: int = 33) -> MaskParams:
    """hcr-mask string (proovread.cfg:235) scaled to min_sr_length (proovread:1702-1705)."""
    L = _abi.lib()
    _setup(L)
    p = MaskParams()
    if hcr_mask is None:
        L.pr_mask_params_default(C.byref(p))
    else:
        _abi.check(L.pr_mask_params_parse(hcr_mask.encode(), min_sr_length, C.byref(p)), "pr_mask_params_parse")
    p.phred_offset = phred_offset
    return p


def pool(seqs: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    off = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    buf = np.frombuffer(b"".join(seqs), np.uint8) if seqs else np.zeros(0, np.uint8)
    return np.ascontiguousarray(buf).copy(), off


def run(seqs: Sequence[bytes], quals: Sequence[bytes], p: MaskParams, ctx: Optional[_abi.Context] = None):
    """Mask reads on the GPU -> (masked sequences, MCR lists [[off, len]], (bpt, bpN))."""
    if len(seqs) != len(quals) or any(len(s) != len(q) for s, q in zip(seqs, quals)):
        raise ValueError("every read needs a quality string of its length")
    L = _abi.lib()
    _setup(L)
    ctx = ctx or _abi.default_context()
    s, off = pool(seqs)
    q, _ = pool(quals)
    n = len(seqs)
    cap = C.c_int64()
    _abi.check(L.pr_mask_bound(C.byref(p), n, off.ctypes.data, C.byref(cap)), "pr_mask_bound")
    out = np.zeros(max(1, len(s)), np.uint8)
    mcr_off = np.zeros(n + 1, np.int64)
    mcr = np.zeros(2 * max(1, cap.value), np.int32)
    n_mcr = np.zeros(max(1, n), np.int32)
    st = np.zeros(2, np.int64)
    _abi.check(L.pr_mask_run(ctx.h, C.byref(p), n, off.ctypes.data, s.ctypes.data, q.ctypes.data, out.ctypes.data,
                             mcr_off.ctypes.data, mcr.ctypes.data, n_mcr.ctypes.data, st.ctypes.data), "pr_mask_run")
    masked: List[bytes] = [out[off[i]:off[i + 1]].tobytes() for i in range(n)]
    mcrs = [mcr[2 * mcr_off[i]:2 * (mcr_off[i] + n_mcr[i])].reshape(-1, 2).tolist() for i in range(n)]
    return masked, mcrs, (int(st[0]), int(st[1]))
