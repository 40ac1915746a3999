"""Probe (GPU box): the 12-byte SMEM-interval build of the seeding core (tools/probe/libprgpu_iv12.so)
on the device vs the same core on the host; which reads differ, whether the difference repeats."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from proovread_amd import _abi  # noqa: E402
if len(sys.argv) > 1:
    _abi.LIBPATH = Path(sys.argv[1])
from proovread_amd import seed  # noqa: E402
from test_seed_gpu import _data, _by_read  # noqa: E402

d, ss, so = _data(12)
n = len(so) - 1
ix = seed.SeedIndex(d.lr_seq, d.lr_off)
ctx = _abi.default_context()
ix.to_gpu(ctx)
for fin in (False, True):
    o = seed.default_opts(fin)
    want, wst = ix.map_device_caps(ss, so, o)
    runs = [ix.map_gpu(ss, so, o, allow_flagged=True) for _ in range(3)]
    wb = _by_read(want, n)
    for k, (got, st) in enumerate(runs):
        gb = _by_read(got, n)
        bad = [i for i in range(n) if gb[i] != wb[i] or st[i] != wst[i]]
        print(f"finish={fin} run{k}: {len(bad)} reads differ, status diffs {int((st != wst).sum())}, "
              f"tasks {len(got)} vs {len(want)}", flush=True)
        if k == 0:
            for i in bad[:6]:
                print(f"  read {i} len {so[i+1]-so[i]} st {st[i]}/{wst[i]}: gpu {len(gb[i])} host {len(wb[i])}")
                for a, b in list(zip(gb[i], wb[i]))[:40]:
                    if a != b:
                        print("    gpu", a, "\n    host", b)
                        break
    same = all(np.array_equal(runs[0][0], r[0]) for r in runs[1:])
    print(f"finish={fin}: GPU runs identical to each other: {same}", flush=True)
