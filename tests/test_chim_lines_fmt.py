"""pr_fmt_chim_lines (the finish task's chimera lines, bam2cns:488, formatted natively) against
the host-language formatting it replaced (f"{id}\\t{from}\\t{to}\\t{npos / ntot:.15g}"), on
random rows with reads without chimeras, unused row slots between reads, and npos / ntot
ratios that print with exponents, as integers, as nan (0 / 0) and as inf (x / 0)."""
import ctypes as C

import numpy as np

from proovread_amd import _abi


def _python_lines(ids, nch, c0, rows):
    idx = np.flatnonzero(nch)
    cnt = nch[idx].astype(np.int64)
    first = np.repeat(c0[idx] - (np.cumsum(cnt) - cnt), cnt)
    r = rows[first + np.arange(int(cnt.sum()))]
    with np.errstate(all="ignore"):
        ratio = (r[:, 2].astype(np.float64) / r[:, 3]).tolist()
    rid = [ids[i] for i in np.repeat(idx, cnt).tolist()]
    return [f"{i}\t{fr}\t{to}\t{x:.15g}" for i, fr, to, x in zip(rid, r[:, 0].tolist(), r[:, 1].tolist(), ratio)]


def test_native_chimera_lines_match_python_formatting():
    L = _abi.lib()
    L.pr_fmt_chim_lines.argtypes = [C.c_int32] + [C.c_void_p] * 5 + [C.POINTER(C.c_void_p), C.POINTER(C.c_int64),
                                                                     C.POINTER(C.c_int64)]
    L.pr_buffer_free.argtypes = [C.c_void_p]
    rng = np.random.default_rng(7)
    n = 4000
    ids = [f"lr{i}_{int(rng.integers(1 << 40))}" for i in range(n)]
    nch = rng.integers(0, 4, n).astype(np.int32)
    nch[::5] = 0
    c0 = np.zeros(n + 1, np.int64)
    np.cumsum(nch + rng.integers(0, 2, n), out=c0[1:])
    rows = rng.integers(0, 20000, (int(c0[-1]) + 1, 4)).astype(np.int32)
    rows[:, 3] = rng.integers(1, 1 << 20, len(rows))
    rows[:, 2] = rng.integers(0, rows[:, 3] + 1)
    rows[::11, 2] = 1                         # 1 / large: exponent form
    rows[::13, 2] = rows[::13, 3]             # 1
    k = c0[np.flatnonzero(nch)[:3]]
    rows[k[0]] = (5, 9, 0, 0)                 # nan
    rows[k[1]] = (5, 9, 3, 0)                 # inf
    want = _python_lines(ids, nch, c0, rows)
    enc = [x.encode() for x in ids]
    off = np.zeros(n + 1, np.int64)
    np.cumsum([len(x) for x in enc], out=off[1:])
    pool = np.frombuffer(b"".join(enc), np.uint8)
    t, ln, nl = C.c_void_p(), C.c_int64(), C.c_int64()
    assert L.pr_fmt_chim_lines(n, pool.ctypes.data, off.ctypes.data, nch.ctypes.data, c0.ctypes.data, rows.ctypes.data,
                               C.byref(t), C.byref(ln), C.byref(nl)) == 0
    got = C.string_at(t.value, ln.value).decode().split("\n")
    L.pr_buffer_free(t)
    assert got[-1] == "" and nl.value == len(want)
    assert got[:-1] == want
    assert any("e-" in x for x in want) and any(x.endswith("\tnan") for x in want) and any(x.endswith("\tinf") for x in want)
