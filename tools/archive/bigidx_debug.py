"""Debug: host vs device k-mer offsets / page splits of the >2^32 test index (GPU box)."""
import ctypes as C
import sys

import numpy as np

sys.path[:0] = ["/root/repo", "/root/repo/tests"]
import test_seed_big_gpu as T  # noqa: E402
from proovread_amd import _abi, seed  # noqa: E402

d, seq, off, na, npad = T.big_long_reads()
L = _abi.lib()
NK = 1 << 24
hk, hs = np.zeros(NK + 1, np.uint64), np.zeros(NK, np.uint64)
dk, ds = np.zeros(NK + 1, np.uint64), np.zeros(NK, np.uint64)
hx = seed.SeedIndex(seq, off)
L.pr_seed_index_koff.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
L.pr_seed_gpu_index_koff.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
L.pr_seed_index_koff(hx.h, hk.ctypes.data, hs.ctypes.data)
ctx = _abi.default_context()
ix = seed.DeviceSeedIndex(ctx, seq, off)
L.pr_seed_gpu_index_koff(ctx.h, dk.ctypes.data, ds.ctypes.data)
print("koff equal", np.array_equal(hk, dk), "ksplit equal", np.array_equal(hs, ds))
bad = np.nonzero(hs != ds)[0]
print("ksplit diffs", len(bad), bad[:10], hs[bad[:10]], ds[bad[:10]], hk[bad[:10]], hk[bad[:10] + 1])
bad = np.nonzero(hk != dk)[0]
print("koff diffs", len(bad), bad[:10], hk[bad[:10]], dk[bad[:10]])
print("host digest  ", hx.digest())
print("device digest", ix.digest())
# the text in numpy: forward reads + SEP, then the reverse complement of the concatenation
n_lr = len(off) - 1
l_pac = int(off[-1])
n = 2 * l_pac + 2 * n_lr
text = np.empty(n, np.uint8)
fw = np.where(seq < 4, seq, 4).astype(np.uint8)
o = 0
for i in range(n_lr):
    a, b = int(off[i]), int(off[i + 1])
    text[o:o + b - a] = fw[a:b]
    text[o + b - a] = 5
    o += b - a + 1
rc = np.where(fw < 4, 3 - fw, 4).astype(np.uint8)[::-1]
o2 = 0
for i in range(n_lr - 1, -1, -1):
    a, b = int(off[i]), int(off[i + 1])
    L = b - a
    text[o:o + L] = rc[l_pac - b:l_pac - a]
    text[o + L] = 5
    o += L + 1
assert o == n
z = np.nonzero(text[:-9] == 0)[0]
cand = []
for p in z:
    if p + 12 <= n and (text[p:p + 9] == 0).all():
        w = text[p:p + 12]
        if (w < 4).all():
            code = 0
            for c in w:
                code = code * 4 + int(c)
            if code < 25:
                cand.append((int(p), code))
    if len(cand) > 20:
        break
print("low-code kmers", cand)
