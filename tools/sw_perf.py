"""Quick SW kernel timing on a synthetic workload (dev tool)."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import ctypes as C
import numpy as np
from proovread_amd import _abi, sw, synth

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
t = time.time()
d = synth.simulate(20261017, int(4_600_000 * scale), int(13800 * scale), 10000, 50, sr_frac=0.3)
print(f"gen {time.time()-t:.1f}s tasks {len(d.t_sr)} LR bases {d.lr_off[-1]}", flush=True)
ctx = _abi.default_context()
L = _abi.lib(); sw._setup(L)
b = d.sw_input().c_batch()
opts = sw.default_opts()
_abi.check(L.pr_sw_upload(ctx.h, C.byref(b)), "upload")
res = sw.SwResult(len(d.t_sr))
for it in range(2):
    t = time.time()
    _abi.check(L.pr_sw_launch(ctx.h, C.byref(opts)), "launch")
    _abi.check(L.pr_sw_download(ctx.h, C.byref(res.c)), "download")
    me, mg, ce, cg = sw.last_timing(ctx)
    print(f"iter {it}: wall {time.time()-t:.3f}s ext {me:.1f}ms glob {mg:.1f}ms cells ext {ce/1e9:.2f}G glob {cg/1e9:.2f}G "
          f"GCUPS ext {ce/me/1e6:.1f} glob {cg/mg/1e6:.1f} frac_valu {(ce*14)/(me*1e-3)/39.3e12:.3f}", flush=True)
print("pass frac", res["pass"].mean(), "status!=0", int((res["status"] != 0).sum()))
