"""Debug (GPU box): the exact layout at world 1 vs the single iteration on a bench-like shard."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo")
from proovread_amd import _abi, cns, iteration, seed, sw, synth, comm as cmod

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 0.2
use_rccl = len(sys.argv) > 2 and sys.argv[2] == "rccl"
d = synth.simulate(20261017, int(4_600_000 * scale), int(13_800 * scale), 10_000, 50.0, sr_frac=0.3)
ctx = _abi.Context(0)
o = seed.default_opts(False)
ix = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
ix.map(d.sr_seq, d.sr_off, o, keep_on_device=True)
opts = sw.default_opts(False)
opts.bin_size, opts.bin_length = 20, 300.0
params = cns.CnsParams(coverage=11.25, use_ref_qual=True)
ref = np.frombuffer(b"ACGTN", np.uint8)[d.lr_seq]
qual = np.full(len(ref), ord("$"), np.uint8)
it = iteration.Iteration(d, lr_qual=qual, ctx=ctx, ref_seq=ref, gpu_seeds=True)
it.launch(opts, params)
a = it.download()
st1 = a["status"].copy()
print("single: ok", int((st1 == 0).sum()), "of", d.n_lr, "alns", it.alignment_stats(), flush=True)
r1 = it.results()
cm = None
if use_rccl:
    cm = cmod.RcclComm(ctx, 0, 1, key="dbg")
ix.map(d.sr_seq, d.sr_off, o, keep_on_device=True)
sh = iteration.ShardSW(ctx, d.sr_seq, d.sr_off, 0, d.n_sr, d.lr_seq, d.lr_off)
ow = iteration.OwnedIteration(ctx, 0, d.n_lr, d.lr_off, ref, qual, d.sr_seq, d.sr_off)
bounds = np.array([0, d.n_lr], np.int64)
from proovread_amd import mask
mp = mask.params("20,41,80,130,60,0.7", 150)
stats = _abi.DevBuffer(ctx, 16)
for rep in range(2):
    sh.launch(opts)
    n = iteration.exchange(ctx, cm, 0, bounds)
    ow.launch(opts, params)
    if len(sys.argv) > 3:   # as bench.py's step
        ow.mask_to(stats.ptr, mp)
        if cm is not None:
            cm.allreduce_dev(stats.ptr, 2)
        ow.sync()
        sw.dominant_kernel(ctx)
        sw.extension_kernels(ctx)
    b = ow.download()
    st2 = b["status"].copy()
    print("rep", rep, "recv", n, "owned: ok", int((st2 == 0).sum()), "alns", ow.alignment_stats(), flush=True)
    bad = np.nonzero(st2 != st1)[0]
    print(" status diffs", len(bad), bad[:10], st2[bad[:10]], flush=True)
    r2 = ow.results()
    diff = [i for i in range(d.n_lr) if (r1[i].seq, r1[i].qual, r1[i].trace) != (r2[i].seq, r2[i].qual, r2[i].trace)]
    print(" result diffs", len(diff), diff[:10], flush=True)
