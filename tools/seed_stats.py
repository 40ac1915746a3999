"""Work counters of the seeding core on a bench-shaped sample (host-only statistics build:
seed.cpp with -DPR_SEED_STATS, tools/seed_stats.cpp).  Prints per-read averages of the
SC_STAT counters in seed_core.h.

    g++ -O2 -std=c++17 -fPIC -shared -pthread -DPR_SEED_STATS -o /tmp/libseedstats.so \
        proovread_amd/csrc/seed.cpp tools/seed_stats.cpp
    python tools/seed_stats.py /tmp/libseedstats.so [n_reads]
"""
import ctypes as C
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from proovread_amd import synth  # noqa: E402
from proovread_amd.seed import SeedOpts, SeedTasks  # noqa: E402

NAMES = {0: "reads", 1: "mems", 2: "hits scanned (chaining)", 3: "occurrences chained", 4: "chain-search steps",
         5: "merges", 6: "new chains", 7: "shifted list elements", 8: "occ() lookups", 9: "occ() hit-list scans",
         10: "hit-list entries scanned", 11: "chains (ncv)", 12: "sum ncv^2", 13: "weight-sort moves",
         14: "chains after weight filter", 15: "tasks out", 16: "smem1 calls", 17: "backward intervals"}

L = C.CDLL(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
L.pr_seed_opts_default.argtypes = [C.POINTER(SeedOpts), C.c_int]
L.pr_seed_index_build.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
L.pr_seed_map.argtypes = [C.c_void_p, C.POINTER(SeedOpts), C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                          C.POINTER(SeedTasks)]
d = synth.simulate(20261015 + 2, 4_600_000, 13_800, 10_000, 50.0, sr_frac=0.3)
seq = np.ascontiguousarray(d.lr_seq, np.uint8)
off = np.ascontiguousarray(d.lr_off, np.int64)
h = C.c_void_p()
assert L.pr_seed_index_build(seq.ctypes.data, off.ctypes.data, len(off) - 1, C.byref(h)) == 0
o = SeedOpts()
L.pr_seed_opts_default(C.byref(o), 0)
L.pr_seed_stat_reset()
sr = np.ascontiguousarray(d.sr_seq[:d.sr_off[n]], np.uint8)
so = np.ascontiguousarray(d.sr_off[:n + 1], np.int64)
out = SeedTasks()
t = time.perf_counter()
assert L.pr_seed_map(h, C.byref(o), sr.ctypes.data, so.ctypes.data, n, 8, C.byref(out)) == 0
dt = time.perf_counter() - t
st = (C.c_ulonglong * 24)()
L.pr_seed_stat_get(st)
r = max(1, st[0])
print(f"{n} reads, {dt:.2f} s on 8 threads (stats build)")
for k, name in NAMES.items():
    print(f"{k:2d} {name:28s} {st[k] / r:12.2f} per read")
