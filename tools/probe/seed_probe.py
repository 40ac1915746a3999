"""Probe (GPU box): GPU seeding of tests/test_seed_gpu.py's data with a given library build, vs the
host emulation; prints timings so a slow or hung kernel shows."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from proovread_amd import _abi  # noqa: E402
if len(sys.argv) > 1:
    _abi.LIBPATH = Path(sys.argv[1])
from proovread_amd import seed  # noqa: E402
from test_seed_gpu import _data  # noqa: E402

d, ss, so = _data(12)
ix = seed.SeedIndex(d.lr_seq, d.lr_off)
ctx = _abi.default_context()
ix.to_gpu(ctx)
for n in (64, 640, len(so) - 1):
    s2, o2 = ss[:so[n]], so[:n + 1]
    want, wst = ix.map_device_caps(s2, o2, seed.default_opts(False))
    t = time.time()
    got, st = ix.map_gpu(s2, o2, seed.default_opts(False), allow_flagged=True)
    print(f"{n} reads: {time.time() - t:.2f} s, equal {np.array_equal(got, want) and np.array_equal(st, wst)}, "
          f"tasks {len(got)} / {len(want)}, pass2 {int((wst != 0).sum())}", flush=True)
