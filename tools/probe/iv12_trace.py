"""Probe (GPU box): read 95 of tests/test_seed_gpu.py's _data(12) alone through the traced
12-byte-interval build (tools/probe/iv12_build.py --trace): the host run of the device path
(pr_seed_map_device_caps) and the GPU (pr_seed_gpu_map) print every bwt_smem1a call's forward
intervals and SMEMs; the two traces and the seeds are written to gpurun_out/ for a diff.

    python tools/probe/iv12_trace.py tools/probe/libiv12_trace.so [read]
"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
if len(sys.argv) > 3 and sys.argv[3] in ("host", "gpu"):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    from proovread_amd import _abi
    _abi.LIBPATH = Path(sys.argv[1])
    from proovread_amd import seed
    from test_seed_gpu import _data
    r = int(sys.argv[2])
    d, ss, so = _data(12)
    q = ss[so[r]:so[r + 1]].copy()
    qo = __import__("numpy").array([0, len(q)], "int64")
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    o = seed.default_opts(False)
    if sys.argv[3] == "host":
        t, st = ix.map_device_caps(q, qo, o, threads=1)
    else:
        ix.to_gpu(_abi.default_context())
        t, st = ix.map_gpu(q, qo, o, allow_flagged=True)
    sys.stdout.flush()
    print("SEEDS", st.tolist(), [tuple(int(v) for v in x) for x in t], flush=True)
    sys.exit(0)
lib, r = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "95"
out = ROOT / "gpurun_out"
out.mkdir(exist_ok=True)
for side in ("host", "gpu"):
    with open(out / f"iv12_{side}.txt", "w") as fh:
        subprocess.run([sys.executable, __file__, lib, r, side], stdout=fh, stderr=subprocess.STDOUT, check=True,
                       timeout=300)
h = (out / "iv12_host.txt").read_text().splitlines()
g = (out / "iv12_gpu.txt").read_text().splitlines()
hs = [x for x in h if x.startswith(("F ", "B ", "  f ", "  m ", "SEEDS"))]
gs = [x for x in g if x.startswith(("F ", "B ", "  f ", "  m ", "SEEDS"))]
print(f"host lines {len(hs)}, gpu lines {len(gs)}")
for k, (a, b) in enumerate(zip(hs, gs)):
    if a != b:
        print(f"first difference at trace line {k}:")
        for x in hs[max(0, k - 6):k + 4]:
            print("  host", x)
        for x in gs[max(0, k - 6):k + 4]:
            print("  gpu ", x)
        break
else:
    print("traces identical" if len(hs) == len(gs) else "one trace is a prefix of the other")
