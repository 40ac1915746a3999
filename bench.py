#!/usr/bin/env python
"""Benchmark of proovread's hot path on MI355X: one correction iteration
(bwa-proovread seed extension + CIGAR, device hand-off, bam2cns consensus) over
a synthetic workload of BASELINE.json configs[1] size per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step = one iteration over the rank's whole batch: SW extension kernels, SW
global/CIGAR kernel, per-read coordinate sort, consensus kernel, the masking of
the corrected reads (SeqFilter --phred-mask) with its {bpt, bpN} statistic
all-reduced across GPUs (RCCL inside libprgpu) as proovread's
mask_shortcut_frac input.  No torch in the process: libprgpu owns the HIP
runtime, the device buffers and the collectives.  Inputs are resident in HBM
before the timed region.  Weak scaling: every rank generates a configs[1]-size
share of the reads (8 ranks ~ configs[2]).

--layout exact (default): the correction loop's own multi-GPU layout
(correct.py; SURVEY.md §8e exact-parity option): every rank
indexes ALL long reads (the ranks' shares all-gathered), seeds and aligns its
short reads against them, and the step sends every reported alignment to the
owner of its long read (device pack + one RCCL all-to-all of device buffers,
pr_aln_exchange) before the owners' -b/-l filter, hand-off and consensus.
--layout shards: every rank indexes only its own long reads (no alignment
exchange; not bit-exact against one index at -D / occurrence caps).

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# INT32 VALU peak: 256 CUs x 64 lanes per clock x 2.4 GHz = 39.3 Tops/s.
# Measured with tools/valu_peak.hip (16 independent v_add_u32/v_max_i32 chains per lane,
# 32 waves/CU): 37.0 Tops/s = 94 % of it (profiles/valu_peak_r01.json) -- integer ops do not
# get the 2-cycle wave64 issue of FP32 (MI355X_MICROARCH.md), so 39.3 is the ceiling.
VALU_PEAK_TOPS = 256 * 64 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0
OPS_PER_CELL = 14   # SURVEY.md §8d canonical int ops per DP cell
# bwa-proovread -b BIN -l LEN of a bwa-sr iteration: BIN = bin-size 20 (proovread.cfg:259-273),
# LEN = BIN x min(--coverage 50, sr-coverage 15) (bin/proovread:1302-1313)
BIN_FILTER = (20, 20.0 * 15.0)
# HBM bytes per launch from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes over this bench
# (tools/pmc_summary.py; MI355X_MICROARCH.md's corrections)
PMC_FILE = "pmc_r04.json"
_JSON_OUT = sys.stdout


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the configs[1] workload per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-lrs-per-worker", type=int, default=256)
    ap.add_argument("--comm", choices=("rccl", "none"), default="rccl",
                    help="rccl: the step all-reduces the device {bpt, bpN} statistic over an RCCL communicator at "
                         "every world size (N=1 included, exactly as N>1 runs it); none: no communicator at N=1")
    ap.add_argument("--layout", choices=("exact", "shards"), default="exact",
                    help="exact: the correction loop's multi-GPU layout (all long reads indexed on every rank, "
                         "alignments all-to-all to the long reads' owners); shards: independent long-read shards")
    ap.add_argument("--seeds", choices=("truth", "host", "gpu"), default="gpu",
                    help="seeds: the product's seeding front end (host path / GPU path; bwa mem seeding "
                         "+ chaining restated; every seed of the kept chains in bwa mode), or the simulation "
                         "truth (one single-seed task per pair); computed before the timed region")
    return ap.parse_args()


def cpu_baseline(d, per_worker: int):
    """The oracle chain (oracle/cpu_bench.py) on the first per_worker x workers long reads, in
    a child process; -> (cpu_baseline JSON object, per-read oracle outputs)."""
    import subprocess
    import tempfile
    workers = min(16, os.cpu_count() or 1)
    n_s = min(d.n_lr, per_worker * workers)
    with tempfile.TemporaryDirectory(prefix="prgpu_bench_") as td:
        npz, out = os.path.join(td, "w.npz"), os.path.join(td, "o.json")
        if d.t_chain is not None:   # bwa mode: every seed of each short read with a seed on the sample
            want = np.zeros(d.n_sr, bool)
            want[d.t_sr[d.t_lr < n_s]] = True
            sel = want[d.t_sr]
            np.savez(npz, lr_seq=d.lr_seq, lr_off=d.lr_off, sr_seq=d.sr_seq, sr_off=d.sr_off,
                     **{k: getattr(d, k)[sel] for k in ("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen",
                                                        "t_chain")})
        else:
            k = int(np.searchsorted(d.t_lr, n_s, side="left"))   # tasks are grouped by long read
            np.savez(npz, lr_seq=d.lr_seq[:int(d.lr_off[n_s])], lr_off=d.lr_off[:n_s + 1], sr_seq=d.sr_seq,
                     sr_off=d.sr_off, t_sr=d.t_sr[:k], t_lr=d.t_lr[:k], t_strand=d.t_strand[:k],
                     t_qbeg=d.t_qbeg[:k], t_rbeg=d.t_rbeg[:k], t_slen=d.t_slen[:k])
        subprocess.run([sys.executable, str(ROOT / "oracle" / "cpu_bench.py"), npz, str(n_s), str(workers), out, "0",
                        str(BIN_FILTER[0]), str(BIN_FILTER[1])], check=True)
        r = json.loads(Path(out).read_text())
    cpu = {"value": round(r["bases"] / r["wall_s"] / 1e6, 4), "unit": "Mbases/s", "cores": r["workers"], "kind": "port",
           "sample": f"first {r['n']} of {d.n_lr} long reads of the same workload ({r['bases']} bases; "
                     + (f"bwa mem per-read alignment of every short read seeded on them, {r['tasks']} seeds"
                        if d.t_chain is not None else f"their {r['tasks']} seed-extension tasks")
                     + f"), SW + consensus C restatement (oracle/), {r['workers']} processes, {r['wall_s']:.1f} s"}
    return cpu, r["results"]


def gather_pool(cm, seq, off):
    """The ranks' read pools back to back in rank order (RCCL all-gather, outside the timed
    region) -> (pool, offsets, global id of this rank's first read)."""
    parts = cm.allgather_bytes(np.ascontiguousarray(seq, np.uint8).tobytes())
    lens = cm.allgather_bytes(np.diff(np.asarray(off, np.int64)).astype(np.int64).tobytes())
    n = [len(x) // 8 for x in lens]
    L = np.concatenate([np.frombuffer(x, np.int64) for x in lens])
    o = np.zeros(len(L) + 1, np.int64)
    np.cumsum(L, out=o[1:])
    return np.frombuffer(b"".join(parts), np.uint8), o, int(sum(n[:cm.rank]))


def check_parity(it, cpu_res):
    """The GPU iteration's corrected reads vs the CPU chain's on the baseline sample, byte for
    byte: FASTQ (sequence + qualities), trace and chimera lines."""
    got = it.results()
    bad = []
    for i, w in enumerate(cpu_res):
        g = got[i]
        rc, fq, tr, ch = w
        ok = rc == 0 and g.status == 0 and g.fastq == fq and g.trace == tr and \
            "".join(l + "\n" for l in g.chim_lines()) == ch
        if not ok:
            bad.append(i)
    return {"checked_reads": len(cpu_res), "mismatches": len(bad), "first_mismatch": bad[:5],
            "against": "oracle chain (bwa mem per-read alignment + SW restatement -> coordinate order -> consensus "
                       "restatement pinned to the reference Perl engine), same seeds"}


def main():
    args = parse()
    # the contract is ONE JSON line on stdout: libraries that print there (RCCL's version
    # banner at communicator init) are sent to stderr, the line goes to the saved stdout
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)
    global _JSON_OUT
    _JSON_OUT = os.fdopen(out_fd, "w")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    from proovread_amd import synth
    # configs[1]: E. coli-size 4.6 Mb genome, 30x 10 kb CLR reads (15 % error: 9 % ins,
    # 4.5 % del, 1.5 % sub), 50x 150 bp short reads, sampled to the iteration's 15x
    # (cov2seqchunker, proovread:2085-2102: int(20*15/50+.5)=6 of 20 chunks).
    gl = int(4_600_000 * args.scale)
    n_lr = int(13_800 * args.scale)
    seed = 20261015 + 2 + 1000 * rank
    t = time.perf_counter()
    d = synth.simulate(seed, gl, n_lr, 10_000, 50.0, sr_frac=0.3)
    gen_s = time.perf_counter() - t
    lr_bases = int(d.lr_off[-1])
    seed_info = None

    def seed_front_end(ctx=None, want_host_copy=True, lr_seq=None, lr_off=None):
        """The front end (bwa-proovread index + mem seeding and chaining) on this rank's reads,
        outside the timed region: the step measures the iteration from resident seeds.
        ctx: index built in HBM and seeding on the GPU, the seeds left in HBM for the
        iteration (no host round trip); with want_host_copy they are also downloaded (CPU
        baseline, and the check against the host path on a sample of reads).  None: host C++
        threads.  lr_seq / lr_off: the long reads indexed (default: this rank's)."""
        from proovread_amd import seed as seeding
        o = seeding.default_opts(False)
        if lr_seq is None:
            lr_seq, lr_off = d.lr_seq, d.lr_off
        t = time.perf_counter()
        if ctx is None:
            ix = seeding.SeedIndex(lr_seq, lr_off)
        else:
            ix = seeding.DeviceSeedIndex(ctx, lr_seq, lr_off)
        t_ix = time.perf_counter() - t
        t = time.perf_counter()
        tasks = None
        if ctx is None:
            tasks = ix.map(d.sr_seq, d.sr_off, o, threads=min(16, os.cpu_count() or 1))
            ms = ix_ms = None
            check = seed_phases = None
        else:
            # steady state: a first, untimed call makes the scratch / output allocations, the
            # timed one is what every later iteration pays
            ix.map(d.sr_seq, d.sr_off, o, keep_on_device=True)
            t = time.perf_counter()
            ix.map(d.sr_seq, d.sr_off, o, keep_on_device=True)
            ms, ix_ms = ix.gpu_ms(), ix.build_ms()
            seed_phases = ix.phase_ms()
        t_map = time.perf_counter() - t
        if ctx is None:
            ix.close()
        elif want_host_copy:
            # the same seeds downloaded (the kernel is deterministic; the device copy stays the
            # iteration's input), and checked against the host path (host index + host seeding)
            # on the first reads of the shard, seed for seed
            tasks, _ = ix.map(d.sr_seq, d.sr_off, o)
            ns = min(d.n_sr, 20_000)
            hx = seeding.SeedIndex(d.lr_seq, d.lr_off)
            want = hx.map(d.sr_seq[:d.sr_off[ns]], d.sr_off[:ns + 1], o, threads=min(16, os.cpu_count() or 1))
            hx.close()
            got = tasks[tasks["sr"] < ns]
            check = {"reads": int(ns), "tasks": int(len(want)), "equal": bool(np.array_equal(got, want))}
            if not check["equal"]:
                raise SystemExit(f"bench: GPU seeding differs from the host path on the first {ns} reads")
        else:
            check = None
        info = {"path": "gpu" if ctx is not None else "host", "index_s": round(t_ix, 3), "map_s": round(t_map, 3),
                "indexed_long_read_bases": int(lr_off[-1]),
                "reads_per_s": round(d.n_sr / t_map, 1), "index_kernel_ms": ix_ms, "kernel_ms": ms,
                "parity_vs_host": check, "kernel_phase_ms_summed_over_waves": seed_phases}
        if tasks is not None:
            info["tasks"] = int(len(tasks))
            info["chains"] = int((tasks["rank"] == 0).sum())
            return synth.with_seeds(d, tasks), info
        return dataclasses.replace(d, t_chain=np.zeros(0, np.int32)), info

    exact = args.layout == "exact"
    if exact and args.seeds != "gpu":
        raise SystemExit("bench: --layout exact seeds on the GPU (--seeds gpu)")
    if args.seeds == "host":
        d, seed_info = seed_front_end()

    # CPU baseline (rank 0, N=1): the oracle chain on a bounded sample of the same workload,
    # in a child process (its fork pool never shares a process with a HIP runtime).  Its
    # per-read outputs are also the parity check of the GPU run below.
    cpu, cpu_res = None, None
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    if want_cpu and args.seeds != "gpu":
        cpu, cpu_res = cpu_baseline(d, args.cpu_lrs_per_worker)

    # GPU: libprgpu only (its own HIP runtime and RCCL); torch is never loaded here
    from proovread_amd import _abi, cns, comm as comm_mod, iteration, sw
    ctx = _abi.Context(local)
    cm = comm_mod.RcclComm.from_env(ctx) if world > 1 or args.comm == "rccl" else None
    # exact layout: the global read set = the ranks' shares in rank order (all-gathered)
    lr_all, lr_off_all, sr_all, sr_off_all, s0 = d.lr_seq, d.lr_off, d.sr_seq, d.sr_off, 0
    gather_s = 0.0
    if exact and world > 1:
        t = time.perf_counter()
        lr_all, lr_off_all, _ = gather_pool(cm, d.lr_seq, d.lr_off)
        sr_all, sr_off_all, s0 = gather_pool(cm, d.sr_seq, d.sr_off)
        gather_s = time.perf_counter() - t
    if args.seeds == "gpu":
        d, seed_info = seed_front_end(ctx, want_host_copy=want_cpu, lr_seq=lr_all, lr_off=lr_off_all)
        if want_cpu:   # the same GPU-made seeds, CPU chain in a child process
            cpu, cpu_res = cpu_baseline(d, args.cpu_lrs_per_worker)
    t_up = time.perf_counter()
    # host -> HBM upload of the reads; GPU seeds stay in HBM (outside the step)
    if exact:
        from proovread_amd import exact_shard as ex
        bounds = ex.lr_bounds(lr_off_all, world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        # the SW batch from the seeding's device pools (no second upload); the consensus reference
        # is the mapped long reads (bwa-sr-1), read from the SW batch on the device
        shard = iteration.ShardSW(ctx, sr_all, sr_off_all, s0, s0 + d.n_sr, lr_all, lr_off_all, device_pools=True)
        qual_all = np.full(len(lr_all), ord("$"), np.uint8)   # raw CLR reads: phred 3
        it = iteration.OwnedIteration(ctx, lo, hi, lr_off_all, None, qual_all, None if world == 1 else sr_all,
                                      sr_off_all)
        own_bases = int(lr_off_all[hi] - lr_off_all[lo])
    else:
        it = iteration.Iteration(d, ctx=ctx, gpu_seeds=args.seeds == "gpu")
        own_bases = lr_bases
    upload_s = time.perf_counter() - t_up
    opts = sw.default_opts(finish=False)
    opts.bin_size, opts.bin_length = BIN_FILTER     # bwa-proovread -b 20 -l 300 (proovread:1302-1313)
    params = cns.CnsParams(coverage=min(50.0, 15.0) * 0.75, use_ref_qual=True)   # proovread:1540-1541
    from proovread_amd import mask
    mparams = mask.params("20,41,80,130,60,0.7", 150)   # hcr-mask of bwa-sr-1 (proovread.cfg:234-242)
    stats = _abi.DevBuffer(ctx, 16)

    def launch():
        if exact:   # SW of the short-read shard, alignments to their owners, owners' consensus
            shard.launch(opts)
            iteration.exchange(ctx, cm, s0, bounds)
        it.launch(opts, params)

    def step():
        launch()
        it.mask_to(stats.ptr, mparams)   # SeqFilter --phred-mask: next reference + {bpt, bpN}
        if cm is not None:
            cm.allreduce_dev(stats.ptr, 2)   # RCCL: global bpt / bpN (mask_shortcut_frac input)
        it.sync()

    def barrier():
        if cm is not None:
            cm.barrier()
        it.sync()

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    ms = np.zeros(4)
    dom_ms, dom_cells = 0.0, 0
    ext_ms, ext_cells, ext_launches = 0.0, 0, 0
    for _ in range(args.steps):
        step()
        ms += np.array(it.timing())
        dm, dc = sw.dominant_kernel(ctx)
        dom_ms += dm
        dom_cells = dc
        xm, xc, xn = sw.extension_kernels(ctx)
        ext_ms += xm
        ext_cells, ext_launches = xc, xn
    barrier()
    el = time.perf_counter() - t0
    e2e_ms = ((seed_info["index_s"] + seed_info["map_s"] + upload_s) * 1e3 + el / args.steps * 1e3
              if seed_info else None)
    if cm is not None:
        el = cm.allreduce_floats([el], comm_mod.RED_MAX)[0]
        total_bases = cm.allreduce_ints([own_bases])[0]
        if e2e_ms is not None:
            e2e_ms = cm.allreduce_floats([e2e_ms], comm_mod.RED_MAX)[0]
    else:
        total_bases = own_bases
    ms /= max(args.steps, 1)
    me, mg, ce, cg = sw.last_timing(ctx)
    bwa_rounds, bwa_ext, bwa_patch = sw.bwa_stats(ctx) if d.t_chain is not None else (0, 0, 0)
    pc = sw.phase_cycles(ctx)
    # one more, untimed step with the consensus kernel's per-phase clock counters on
    os.environ["PRGPU_CNS_PROF"] = "1"
    step()
    os.environ.pop("PRGPU_CNS_PROF")
    cns_phases = it.cns_phase_ms()
    a = it.download()
    ok = int((a["status"] == 0).sum())
    bpt, bpn = (int(x) for x in stats.download(np.int64))
    parity = check_parity(it, cpu_res) if cpu_res is not None else None
    if rank != 0:
        if cm is not None:
            cm.close()
        return
    value = total_bases * args.steps / el / 1e6
    cells = ce + cg
    dom_ms /= max(args.steps, 1)
    dom_tops = dom_cells * OPS_PER_CELL / (dom_ms * 1e-3) / 1e12
    ext_ms /= max(args.steps, 1)
    ext_tops = ext_cells * OPS_PER_CELL / (ext_ms * 1e-3) / 1e12 if ext_ms > 0 else 0.0
    # pileup kernel: algorithmic bytes (SURVEY.md §8d model) / kernel time
    n_aln, sum_ncig, sum_lseq = it.alignment_stats()
    cns_bytes = sum_lseq + 4 * sum_ncig + 16 * n_aln + own_bases * (2 + 2 + 6 * 4 * 2)
    # HBM bytes per launch from the PMC FETCH_SIZE / WRITE_SIZE passes of this bwa-mode step
    # (tools/r04_final.sh -> tools/pmc_summary.py -> profiles/pmc_r04.json)
    prof = ROOT / "profiles" / PMC_FILE
    traffic = traffic_cns = traffic_ext = None
    if prof.exists():
        try:
            pm = json.loads(prof.read_text())
            traffic = next((v.get("hbm_bytes_per_launch") for k, v in pm.items() if k.startswith("sw_global_pk_kernel<40")),
                           None)
            traffic_cns = next((v.get("hbm_bytes_per_launch") for k, v in pm.items() if k.startswith("cns_lr_kernel")), None)
            traffic_ext = {k: v.get("hbm_bytes_per_launch") for k, v in pm.items() if k.startswith("sw_ext_")}
        except Exception:
            traffic = traffic_cns = traffic_ext = None
    ref_cpu = None   # the reference's own Perl consensus, timed in the build container
    rp = ROOT / "profiles" / "r03_reference_cpu_consensus.json"
    if rp.exists():
        try:
            r3 = json.loads(rp.read_text())
            rpl = r3["reference_perl"]
            ref_cpu = {"value": rpl["Mbases_per_s"], "unit": "Mbases/s", "cores": rpl["processes"], "kind": "reference",
                       "scope": "consensus only, build container", "cpu": r3["host"]["cpu"],
                       "sample": r3["workload"] + f"; {rpl['engine']}; {rpl['wall_s']} s wall",
                       "source": "profiles/r03_reference_cpu_consensus.json (tools/time_reference_r03.py)"}
        except Exception:
            ref_cpu = None
    out = {
        "metric": "corrected long-read Mbases/sec per node",
        "value": round(value, 3),
        "unit": "Mbases/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic: iid genome, CLR-like long reads, 150 bp short reads, seeds from "
                + ("the simulation truth" if args.seeds == "truth" else f"the {args.seeds} seeding path"),
        "config": {
            "workload": "configs[1] per GPU: 4.6 Mb genome, 13,800 x 10 kb long reads (30x, 15% error), "
                        "50x 2x150 short reads sampled to 15x for one bwa-sr iteration",
            "genome_bp": gl, "long_reads_per_gpu": d.n_lr, "long_read_bases_per_gpu": lr_bases,
            "short_reads_per_gpu": d.n_sr, "seeds_per_gpu": it.n_task, "task": "bwa-sr-1",
            "coverage_cap": params.coverage,
            "parallelism": (f"exact-parity layout x{world}: every rank indexes all {len(lr_off_all) - 1} long reads "
                            f"({int(lr_off_all[-1])} bases), aligns its short reads, alignments all-to-all to the "
                            f"long reads' owners over RCCL (pr_aln_exchange)" if exact else f"long-read shards x{world}"),
            "layout": args.layout,
        },
        "sw_gcups": round(cells / ((ms[0] + ms[1]) * 1e-3) / 1e9, 2),
        # bwa mode: mem_chain2aln rounds, seeds extended (first seeds of every chain + the ones the
        # containment test sends), mem_patch_reg global scores; alignments reported
        "bwa": {"rounds": bwa_rounds, "seeds_extended": bwa_ext, "patches": bwa_patch},
        "stage_ms": {"sw_extend": round(ms[0], 3), "sw_global_cigar": round(ms[1], 3),
                     "handoff_sort": round(ms[2], 3), "consensus": round(ms[3], 3)},
        "cigar_kernel_phase_share": {k: round(v / max(sum(pc), 1), 3) for k, v in
                                     zip(("masks", "dp", "backtrack", "emit"), pc)},
        "consensus_phase_ms_summed_over_workgroups": {k: round(v, 1) for k, v in cns_phases.items()},
        "roofline": {
            "kernel": "sw_global_pk_kernel<40> (ksw_global2 CIGAR pass + backtrack, packed int16, two tasks per lane)",
            "bound": "valu",
            "achieved": round(dom_tops, 3),
            "peak": round(VALU_PEAK_TOPS, 2),
            "unit": "TOP/s (int32)",
            "frac": round(dom_tops / VALU_PEAK_TOPS, 4),
            "traffic": traffic,
            "launch_ms": round(dom_ms, 3),
            "cells_per_launch": int(dom_cells),
            "ops_per_cell": OPS_PER_CELL,
            "peak_packed_int16": round(2 * VALU_PEAK_TOPS, 2),
            "frac_of_packed_int16_peak": round(dom_tops / (2 * VALU_PEAK_TOPS), 4),
        },
        "roofline_consensus": {
            "kernel": "cns_lr_kernel (bin cap + pileup + argmax, one long read per workgroup)", "bound": "hbm",
            "achieved": round(cns_bytes / (ms[3] * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(cns_bytes / (ms[3] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": int(cns_bytes),
            "alignments": int(n_aln), "traffic": traffic_cns,
        },
        "roofline_extension": {
            "kernels": "every ksw_extend2 DP launch of the step (sw_ext_pk_kernel<40>, sw_ext_phase_kernel<*>, wide), "
                       "all bwa-mode rounds, both sides and band tries",
            "bound": "valu", "achieved": round(ext_tops, 3), "peak": round(VALU_PEAK_TOPS, 2), "unit": "TOP/s (int32)",
            "frac": round(ext_tops / VALU_PEAK_TOPS, 4), "summed_launch_ms": round(ext_ms, 3),
            "launches": ext_launches, "cells": int(ext_cells), "ops_per_cell": OPS_PER_CELL,
            "frac_of_packed_int16_peak": round(ext_tops / (2 * VALU_PEAK_TOPS), 4),
            "traffic_per_launch": traffic_ext,
        },
        "cpu_baseline": cpu,
        "cpu_baseline_reference": ref_cpu,
        "comm": "rccl" if cm is not None else "none",
        "seeding": seed_info,
        # one whole bwa-sr iteration as proovread runs it, wall clock: index build + seeding
        # (bwa-proovread index / mem front end; seeds left in HBM) + upload + the timed step
        "iteration_end_to_end_ms": round(e2e_ms, 1) if e2e_ms is not None else None,
        # whole-iteration throughput (index + seeding + upload + step, max over ranks): the rate of a
        # bwa-sr task as the loop runs it; `value` is the step alone (inputs and seeds resident)
        "value_iteration": round(total_bases / (e2e_ms * 1e-3) / 1e6, 3) if e2e_ms else None,
        "read_gather_ms": round(gather_s * 1e3, 1),
        "upload_ms": round(upload_s * 1e3, 1),
        "gen_s": round(gen_s, 1),
        "reads_ok": ok,
        "iteration_stat": {"bpt": bpt, "bpN": bpn, "masked_frac": round(bpn / bpt, 4) if bpt else None},
        "parity": parity,
    }
    print(json.dumps(out), file=_JSON_OUT, flush=True)
    if cm is not None:
        cm.close()
    if parity is not None and parity["mismatches"]:
        raise SystemExit(f"bench: {parity['mismatches']} of {parity['checked_reads']} reads differ from the CPU chain")


if __name__ == "__main__":
    main()
