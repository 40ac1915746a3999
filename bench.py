#!/usr/bin/env python
"""Benchmark of proovread's hot path on MI355X: one correction iteration
(bwa-proovread seed extension + CIGAR, device hand-off, bam2cns consensus) over
a synthetic workload of BASELINE.json configs[1] size per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step = one iteration over the rank's whole batch (every long read of the
shard, every seed-extension task): SW extension kernel, SW global/CIGAR
kernel, per-read coordinate sort, consensus kernel, and the per-iteration
statistic all-reduced across GPUs (RCCL) as proovread's masked-fraction input.
Inputs are resident in HBM before the timed region.  Long reads shard across
GPUs with no data-path collective (weak scaling: every rank holds a
configs[1]-size shard; 8 ranks ~ configs[2]).

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
from __future__ import annotations

import argparse
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the configs[1] workload per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-lrs-per-worker", type=int, default=256)
    ap.add_argument("--seeds", choices=("truth", "host", "gpu"), default="host",
                    help="task list: the product's seeding front end (host path / GPU path; bwa mem seeding "
                         "+ chaining restated), or the simulation truth; computed before the timed region")
    return ap.parse_args()


def main():
    args = parse()
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

    def seed_front_end(ctx=None):
        """The front end (bwa-proovread mem seeding + chaining) on this rank's reads, outside
        the timed region: the step measures the iteration from resident tasks."""
        from proovread_amd import seed as seeding
        t = time.perf_counter()
        ix = seeding.SeedIndex(d.lr_seq, d.lr_off)
        t_ix = time.perf_counter() - t
        t = time.perf_counter()
        if ctx is None:
            tasks = ix.map(d.sr_seq, d.sr_off, seeding.default_opts(False), threads=min(16, os.cpu_count() or 1))
            ms = None
        else:
            ix.to_gpu(ctx)
            tasks, _ = ix.map_gpu(d.sr_seq, d.sr_off, seeding.default_opts(False))
            ms = ix.gpu_ms()
        t_map = time.perf_counter() - t
        ix.close()
        info = {"path": "gpu" if ctx is not None else "host", "index_s": round(t_ix, 2), "map_s": round(t_map, 2),
                "reads_per_s": round(d.n_sr / t_map, 1), "kernel_ms": ms, "tasks": int(len(tasks))}
        return synth.with_seeded_tasks(d, tasks), info

    if args.seeds == "host":   # before the CPU baseline, which then runs on the same tasks
        d, seed_info = seed_front_end()

    # CPU baseline (rank 0, N=1): the oracle chain on a bounded sample of the same
    # workload, before this process touches the GPU (the pool forks).
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, str(ROOT / "oracle"))
        import cpu_chain
        workers = min(16, os.cpu_count() or 1)
        n_s = min(d.n_lr, args.cpu_lrs_per_worker * workers)
        wall, bases, res, nw = cpu_chain.run_sample(d, range(n_s), workers=workers)
        cpu = {"value": round(bases / wall / 1e6, 4), "unit": "Mbases/s", "cores": nw, "kind": "port",
               "sample": f"first {n_s} of {d.n_lr} long reads of the same workload ({bases} bases, their "
                         f"{int(d._task_off[n_s])} seed-extension tasks), SW + consensus C restatement, "
                         f"{nw} processes, {wall:.1f} s"}

    import torch
    import torch.distributed as dist
    from proovread_amd import _abi, cns, iteration, sw
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    ctx = _abi.Context(local)
    if args.seeds == "gpu":   # after the CPU baseline (its worker pool forks before any GPU use)
        d, seed_info = seed_front_end(ctx)
        if cpu is not None:
            cpu["sample"] += " (simulation-truth tasks)"
    it = iteration.Iteration(d, ctx=ctx)
    opts = sw.default_opts(finish=False)
    params = cns.CnsParams(coverage=min(50.0, 15.0) * 0.75, use_ref_qual=True)   # proovread:1540-1541
    stats = torch.zeros(2, dtype=torch.int64, device=dev)

    def step():
        it.launch(opts, params)
        it.stats_to(stats.data_ptr())
        it.sync()
        if world > 1:
            dist.all_reduce(stats)   # RCCL: global corrected / high-quality bases

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ms = np.zeros(4)
    dom_ms, dom_cells = 0.0, 0
    for _ in range(args.steps):
        step()
        ms += np.array(it.timing())
        dm, dc = sw.dominant_kernel(ctx)
        dom_ms += dm
        dom_cells = dc
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        te = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        el = float(te.item())
        tb = torch.tensor([lr_bases], dtype=torch.int64, device=dev)
        dist.all_reduce(tb)
        total_bases = int(tb.item())
    else:
        total_bases = lr_bases
    ms /= max(args.steps, 1)
    me, mg, ce, cg = sw.last_timing(ctx)
    pc = sw.phase_cycles(ctx)
    a = it.download()
    cns_phases = it.cns_phase_ms()
    ok = int((a["status"] == 0).sum())
    hq = stats.cpu().tolist()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    value = total_bases * args.steps / el / 1e6
    cells = ce + cg
    dom_ms /= max(args.steps, 1)
    dom_tops = dom_cells * OPS_PER_CELL / (dom_ms * 1e-3) / 1e12
    # pileup kernel: algorithmic bytes (SURVEY.md §8d model) / kernel time
    n_aln, sum_ncig, sum_lseq = it.alignment_stats()
    cns_bytes = sum_lseq + 4 * sum_ncig + 16 * n_aln + lr_bases * (2 + 2 + 6 * 4 * 2)
    prof = ROOT / "profiles" / "pmc_r01.json"
    traffic = None
    if prof.exists():
        try:
            traffic = json.loads(prof.read_text()).get("sw_global_pk_kernel<40>", {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
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
            "short_reads_per_gpu": d.n_sr, "sw_tasks_per_gpu": int(len(d.t_sr)), "task": "bwa-sr-1",
            "coverage_cap": params.coverage, "parallelism": f"long-read shards x{world}",
        },
        "sw_gcups": round(cells / ((ms[0] + ms[1]) * 1e-3) / 1e9, 2),
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
            "alignments": int(n_aln),
        },
        "cpu_baseline": cpu,
        "seeding": seed_info,
        "gen_s": round(gen_s, 1),
        "reads_ok": ok,
        "iteration_stat": {"corrected_bases": hq[0], "phred_ge20_bases": hq[1]},
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
