"""Final quality-trim windows (`SeqFilter --trim-win`, proovread.cfg:152-155) through
libprgpu.so's host pr_trim_windows (Fastq::Seq::qual_window, Seq.pm:1064-1160)."""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _abi


class TrimParams(C.Structure):
    _fields_ = [("size", C.c_int32), ("soft", C.c_int32), ("hard", C.c_int32), ("min_len", C.c_int32),
                ("phred_offset", C.c_int32)]


def _setup(L):
    if getattr(L, "_trim_ready", False):
        return
    L.pr_trim_params_default.argtypes = [C.POINTER(TrimParams)]
    L.pr_trim_params_parse.argtypes = [C.c_char_p, C.POINTER(TrimParams)]
    L.pr_trim_bound.argtypes = [C.POINTER(TrimParams), C.c_int32, C.c_void_p, C.POINTER(C.c_int64)]
    L.pr_trim_windows.argtypes = [C.POINTER(TrimParams), C.c_int32] + [C.c_void_p] * 5 + [C.c_int]
    L._trim_ready = True


def params(trim_win: Optional[str] = None, phred_offset: int = 33) -> TrimParams:
    L = _abi.lib()
    _setup(L)
    p = TrimParams()
    if trim_win is None:
        L.pr_trim_params_default(C.byref(p))
    else:
        _abi.check(L.pr_trim_params_parse(trim_win.encode(), C.byref(p)), "pr_trim_params_parse")
    p.phred_offset = phred_offset
    return p


def windows(quals: Sequence[bytes], p: TrimParams, threads: int = 0) -> List[List[Tuple[int, int]]]:
    """[(offset, length)] windows of every quality string, in order."""
    L = _abi.lib()
    _setup(L)
    n = len(quals)
    off = np.zeros(n + 1, np.int64)
    np.cumsum([len(q) for q in quals], out=off[1:])
    buf = np.frombuffer(b"".join(quals), np.uint8).copy() if n else np.zeros(1, np.uint8)
    cap = C.c_int64()
    _abi.check(L.pr_trim_bound(C.byref(p), n, off.ctypes.data, C.byref(cap)), "pr_trim_bound")
    woff = np.zeros(n + 1, np.int64)
    win = np.zeros(2 * max(1, cap.value), np.int32)
    nw = np.zeros(max(1, n), np.int32)
    _abi.check(L.pr_trim_windows(C.byref(p), n, off.ctypes.data, buf.ctypes.data, woff.ctypes.data,
                                 win.ctypes.data, nw.ctypes.data, threads), "pr_trim_windows")
    return [[(int(win[2 * k]), int(win[2 * k + 1])) for k in range(woff[i], woff[i] + nw[i])] for i in range(n)]
