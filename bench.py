#!/usr/bin/env python
"""Benchmark of proovread's hot path on MI355X: the whole sr-noccs correction run per step --
read-long's output restored in HBM, then bwa-sr-1 .. bwa-sr-N with mask_shortcut_frac and
bwa-sr-finish (bin/proovread:705-905, 2026-2047) -- over a synthetic workload of BASELINE.json
configs[1] size per GPU; beside it the rate of one bwa-sr-1 task (value_task).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One step = one correction run as proovread makes it (correct.run_tasks on correct.GpuStages, the
loop's multi-GPU layout; SURVEY.md §8e exact-parity option): the long-read set back
to read-long's output (pr_lrset_restore, device to device), then per task

  sampling  SeqChunker's chunks of the short-read stream for the task's coverage
            (cov2seqchunker, bin/proovread:2085-2102), gathered on the device from the
            resident short reads (every rank its contiguous share of the sample)
  index     pr_lrset_index: the seed index of ALL long reads' mapping reference (the finish
            task: the reads), from the resident set in HBM
  seeding   pr_seed_gpu_map_sampled: bwa-proovread mem's seeding and chaining, seeds left in HBM
  SW        pr_sw_upload_gpu_seeds + pr_sw_launch: bwa mode over every seed of the kept chains
  exchange  pr_aln_exchange: every reported alignment to the owner of its long read (RCCL
            all-to-all; at N = 1 the identity)
  consensus pr_iter_upload_owned + pr_iter_launch: the -b/-l filter, hand-off and consensus
  mask      pr_iter_mask + the {bpt, bpN} all-reduce -> mask_shortcut_frac (regular tasks)
  commit    pr_lrset_commit: the corrected (and masked) reads replace the set, all-gathered
            across the ranks

`value` = the corrected long-read bases of the whole job per second of the run.  `value_task`
repeats bwa-sr-1 alone on the raw reads (the round-5 headline's scope, commit DRY).

Every rank generates the SAME global dataset (one genome, one long-read set, one 50x short-read
run in sequencer order -- unsorted over the genome): configs[1] x N (weak scaling: each rank owns
13,800 long reads and aligns 1/N of every task's sample; at N > 1 about (N-1)/N of its alignments
belong to another rank's long reads and cross xGMI).  Inputs are resident in HBM before the
timed region; no torch in the process (libprgpu owns the HIP runtime and RCCL).

Prints ONE JSON line on rank 0 (see DESIGN.md §5 for every field).
"""
from __future__ import annotations

import argparse
import ctypes as C
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
SEED = 20261015 + 2   # 20261015 + config number
# configs[1] per GPU: 4.6 Mb genome, 13,800 x 10 kb CLR reads (30x, 15 % error), 50x 150 bp
# short reads, sampled per task by SeqChunker (cov2seqchunker, proovread:2085-2102: 6 of 20
# chunks for the regular tasks' 15x, 12 of 20 for the finish task's 30x)
GENOME, N_LR, SR_COV = 4_600_000, 13_800, 50.0
# bwa-proovread -b BIN -l LEN of a bwa-sr iteration: BIN = bin-size 20 (proovread.cfg:259-273),
# LEN = BIN x min(--coverage 50, sr-coverage 15) (bin/proovread:1302-1313)
BIN_FILTER = (20, 20.0 * 15.0)
HCR_MASK = "20,41,80,130,60,0.7"   # hcr-mask of bwa-sr-1 (proovread.cfg:234-242)
# HBM bytes per launch from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes over this bench
# (tools/pmc_summary.py; MI355X_MICROARCH.md's corrections)
PMC_FILE = "pmc_traffic.json"   # (repo root: profiles/ does not travel to the GPU box)
_JSON_OUT = sys.stdout


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the configs[1] workload per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--loop-only", action="store_true",
                    help="profiling: the correction runs only (no value_task phase, no CPU baseline)")
    ap.add_argument("--task-only", action="store_true",
                    help="profiling: one untimed correction run, then the timed bwa-sr-1 tasks (value_task, rooflines); "
                         "value is then not a measurement (rocprof / PMC passes of the roofline kernels)")
    ap.add_argument("--cpu-lrs-per-worker", type=int, default=256)
    ap.add_argument("--comm", choices=("rccl", "none"), default="rccl",
                    help="rccl: the step all-reduces the device {bpt, bpN} statistic over an RCCL communicator at "
                         "every world size (N=1 included, exactly as N>1 runs it); none: no communicator at N=1")
    return ap.parse_args()


def host_cpu() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(d, per_worker: int):
    """The oracle chain (oracle/cpu_bench.py) on the first per_worker x workers long reads, in
    a child process; -> (cpu_baseline JSON object, per-read oracle outputs)."""
    import subprocess
    import tempfile
    workers = min(16, os.cpu_count() or 1)
    n_s = min(d.n_lr, per_worker * workers)
    with tempfile.TemporaryDirectory(prefix="prgpu_bench_") as td:
        npz, out = os.path.join(td, "w.npz"), os.path.join(td, "o.json")
        # bwa mode: every seed of each short read with a seed on the sample
        want = np.zeros(d.n_sr, bool)
        want[d.t_sr[d.t_lr < n_s]] = True
        sel = want[d.t_sr]
        np.savez(npz, lr_seq=d.lr_seq, lr_off=d.lr_off, sr_seq=d.sr_seq, sr_off=d.sr_off,
                 **{k: getattr(d, k)[sel] for k in ("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen",
                                                    "t_chain")})
        subprocess.run([sys.executable, str(ROOT / "oracle" / "cpu_bench.py"), npz, str(n_s), str(workers), out, "0",
                        str(BIN_FILTER[0]), str(BIN_FILTER[1])], check=True)
        r = json.loads(Path(out).read_text())
    cpu = {"value": round(r["bases"] / r["wall_s"] / 1e6, 4), "unit": "Mbases/s", "cores": r["workers"], "kind": "port",
           "cpu": host_cpu(), "compare_with": "value_task (one bwa-sr-1 task)",
           "sample": f"one bwa-sr-1 task on the first {r['n']} of {d.n_lr} long reads of the same workload "
                     f"({r['bases']} bases; bwa mem per-read alignment of every short read seeded on them, "
                     f"{r['tasks']} seeds), SW + consensus C restatement (oracle/), {r['workers']} processes, "
                     f"{r['wall_s']:.1f} s; the seeding, index build and masking are NOT included (the GPU "
                     f"value_task includes them)"}
    return cpu, r["results"]


def check_parity(it, cpu_res):
    """The GPU task's corrected reads vs the CPU chain's on the baseline sample, byte for byte:
    FASTQ (sequence + qualities), trace and chimera lines."""
    got = it.results_range(0, len(cpu_res))
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


def reference_cpu():
    """The reference's own Perl consensus (lib/Sam/Seq.pm), timed in the build container where
    /root/reference exists (tools/time_reference_r03.py); the record travels with the tree."""
    rp = ROOT / "baselines" / "reference_cpu_consensus_r03.json"
    if not rp.exists():
        return None
    try:
        r3 = json.loads(rp.read_text())
        rpl = r3["reference_perl"]
        return {"value": rpl["Mbases_per_s"], "unit": "Mbases/s", "cores": rpl["processes"], "kind": "reference",
                "scope": "consensus only (bam2cns over Sam::Seq), build container", "cpu": r3["host"]["cpu"],
                "sample": r3["workload"] + f"; {rpl['engine']}; {rpl['wall_s']} s wall",
                "source": "baselines/reference_cpu_consensus_r03.json (tools/time_reference_r03.py)"}
    except Exception:
        return None


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
    gl = int(GENOME * args.scale * world)
    n_lr = int(N_LR * args.scale * world)
    n_sr = int(round(SR_COV * gl / 150))
    t = time.perf_counter()
    threads = max(1, min(16, (os.cpu_count() or 1) // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", world)))))
    d = synth.simulate_reads(SEED, gl, n_lr, 10_000, n_sr, threads=threads)   # the same on every rank
    gen_s = time.perf_counter() - t

    from proovread_amd import _abi, cns, comm as comm_mod, control, correct, exact_shard as ex, seed, sw
    from proovread_amd import tasks as T
    ctx = _abi.Context(local)
    cm = comm_mod.RcclComm.from_env(ctx) if world > 1 or args.comm == "rccl" else None
    L = _abi.lib()
    from proovread_amd import iteration
    iteration._setup(L)
    seed._setup(L)
    # resident inputs: every long read (ASCII + '$' qualities: raw CLR reads, phred 3) and the
    # whole 50x short-read run on every rank
    t_up = time.perf_counter()
    ascii_pool = np.frombuffer(b"ACGTN", np.uint8)[d.lr_seq[:int(d.lr_off[-1])]]
    stages = correct.GpuStages(ctx)
    stages.load(correct.LongReads([f"lr{i}" for i in range(n_lr)],
                                  pools=(ascii_pool, d.lr_off, np.full(len(ascii_pool), ord("$"), np.uint8))))
    del ascii_pool
    stages.snapshot()                      # read-long's output: every step restarts from it
    srs = correct.ShortReads.from_pool(d.sr_seq[:int(d.sr_off[-1])], d.sr_off)
    stages.load_short_reads(srs)
    upload_s = time.perf_counter() - t_up
    lrs = stages.lrs
    lr_off = d.lr_off
    bounds = ex.lr_bounds(lr_off, world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    own_bases = int(lr_off[hi] - lr_off[lo])
    cfg = correct.LoopConfig(coverage=50.0, exact_layout=True)
    mode = "sr-noccs"
    loop_tasks = list(T.MODE_TASKS[mode][1:])   # after read-long (proovread.cfg:119)
    min_sr = 150

    # ------------------------------------------------------------------ the whole run (value)
    def loop_step():
        stages.restore()
        chim, _, log = correct.run_tasks(stages, srs, loop_tasks, cfg, mode, min_sr, True, cm)
        return chim, log

    def digest(chim):
        import hashlib
        off, sq, ql, _ = lrs.download(seq=True, qual=True)
        h = hashlib.sha256(off.tobytes())
        h.update(sq.tobytes())
        h.update(ql.tobytes())
        h.update("".join(chim).encode())
        return h.hexdigest()

    first_digest = None
    for k in range(0 if args.task_only else args.warmup):
        chim, _ = loop_step()
        if k == 0:
            first_digest = digest(chim)
    if cm is not None:
        cm.barrier()
    _abi.check(L.pr_ctx_sync(ctx.h), "pr_ctx_sync")
    t0 = time.perf_counter()
    dev0 = stages.device_ms
    logs = []
    chim = []
    for _ in range(0 if args.task_only else args.steps):   # (task-only: no correction run at all)
        chim, log = loop_step()
        logs.append(log)
    logs = logs or [[]]
    if cm is not None:
        cm.barrier()
    _abi.check(L.pr_ctx_sync(ctx.h), "pr_ctx_sync")
    el = time.perf_counter() - t0
    loop_dev_ms = (stages.device_ms - dev0) / max(args.steps, 1)
    last_digest = digest(chim) if not args.task_only else None
    n_chim = len(chim)
    if cm is not None:
        el = cm.allreduce_floats([el], comm_mod.RED_MAX)[0]
        total_bases = cm.allreduce_ints([own_bases])[0]
    else:
        total_bases = own_bases
    log = logs[-1]
    loop_rows = [{"task": e.task, "short_reads": e.n_sr, "seeds_rank": e.n_tasks, "wall_ms": e.wall_ms,
                  "device_ms": e.device_ms, "masked_frac": None if e.masked_frac is None else round(e.masked_frac, 4),
                  "shortcut": e.shortcut, "stage_event_ms": e.stage_ms, "part_wall_ms": e.part_ms, "pre_ms": e.pre_ms} for e in log]
    same_tasks = all([e.task for e in lg] == [e.task for e in log] for lg in logs)

    if args.loop_only:
        if rank == 0:
            print(json.dumps({"metric": "corrected long-read Mbases/sec per node", "value": round(
                total_bases * args.steps / el / 1e6, 3), "unit": "Mbases/s", "n_gpus": world, "steps": args.steps,
                "ms_per_step": round(el / args.steps * 1e3, 3), "loop": {"tasks": loop_rows,
                                                                      "device_ms": round(loop_dev_ms, 1),
                                                                      "chimera_lines": n_chim,
                                                                      "final_reads_sha256": last_digest},
                "last_task_seeding_phases": seed._phase_ms(L, ctx),
                # (with PRGPU_CNS_PROF=1 in the environment: the finish task's consensus phases)
                "last_task_consensus_phases": stages.last_iteration.cns_phase_ms()
                if os.environ.get("PRGPU_CNS_PROF") else None}),
                  file=_JSON_OUT, flush=True)
        if cm is not None:
            cm.close()
        return
    # ------------------------------------------------------------------ one bwa-sr-1 task (value_task)
    sampler = control.Sampler(sampling=cfg.sampling)
    rg1, off1 = srs.sample_ranges(sampler.cov2seqchunker(cfg.coverage, T.sr_coverage("bwa-sr-1")))
    n1 = len(off1) - 1
    s0, s1 = ex.sr_range(n1, world, rank)
    params1 = cns.CnsParams(coverage=min(50.0, 15.0) * 0.75, use_ref_qual=True, max_ins_length=0)   # :1540-1541
    sopts = seed.default_opts(False)
    stages.restore()
    wall = {}

    def task_step(dry=True):
        t0 = time.perf_counter()
        stages.task("bwa-sr-1", None, off1, params1, BIN_FILTER, cm, True, (HCR_MASK, min_sr), sr_ranges=rg1,
                    dry=dry)
        wall["task"] = wall.get("task", 0.0) + time.perf_counter() - t0
        return stages.last_iteration

    for _ in range(args.warmup):
        task_step()
    wall.clear()
    if cm is not None:
        cm.barrier()
    _abi.check(L.pr_ctx_sync(ctx.h), "pr_ctx_sync")
    t0 = time.perf_counter()
    ev = np.zeros(6)
    dom_ms = dom_cells = ext_ms = ext_cells = ext_launches = 0
    sw_stage_ms = sw_cells = 0.0
    bwa_ms = np.zeros(3)   # walk, main-stream final passes, early final pass (HIP events)
    for _ in range(args.steps):
        it = task_step()
        ev += np.array([lrs_index_ms(L, ctx), seed._last_ms(L.pr_seed_gpu_last_ms, ctx), *it.timing()])
        dm, dom_cells = sw.dominant_kernel(ctx)
        dom_ms += dm
        xm, ext_cells, ext_launches = sw.extension_kernels(ctx)
        ext_ms += xm
        me, mg, ce, cg = sw.last_timing(ctx)
        sw_stage_ms += me + mg
        sw_cells += ce + cg
        bwa_ms += np.array(sw.bwa_timing(ctx))
    if cm is not None:
        cm.barrier()
    _abi.check(L.pr_ctx_sync(ctx.h), "pr_ctx_sync")
    el_task = time.perf_counter() - t0
    if cm is not None:
        el_task = cm.allreduce_floats([el_task], comm_mod.RED_MAX)[0]
    K = max(args.steps, 1)
    ev /= K
    task_wall = {k: round(v / K * 1e3, 2) for k, v in wall.items()}
    n_seeds = seed._count(L, ctx)
    bwa_rounds, bwa_ext, bwa_patch = sw.bwa_stats(ctx)
    bwa_ms /= K
    na_rep = C.c_int64()
    _abi.check(L.pr_sw_aln_count(ctx.h, C.byref(na_rep)), "pr_sw_aln_count")
    pc = sw.phase_cycles(ctx)
    n_recv = it.n_task
    n_aln, sum_ncig, sum_lseq = it.alignment_stats()
    # one more, untimed task with the consensus kernel's per-phase clock counters on
    os.environ["PRGPU_CNS_PROF"] = "1"
    it = task_step()
    os.environ.pop("PRGPU_CNS_PROF")
    cns_phases = it.cns_phase_ms()
    seed_phases = seed._phase_ms(L, ctx)
    status = it.statuses()
    ok = int((status == 0).sum())
    # checks outside the timed region (rank 0 at N = 1): GPU seeds = the host seeding path on
    # 20 k reads of the task's sample; the CPU baseline (oracle chain) on a bounded sample,
    # whose per-read outputs are also the parity check of the GPU task
    cpu = cpu_res = parity = seed_check = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import dataclasses
        sr1 = np.ascontiguousarray(srs.gather(rg1), np.uint8)
        dt = dataclasses.replace(d, sr_seq=sr1, sr_off=np.ascontiguousarray(off1, np.int64))
        gpu_tasks, gst = seed._map_gpu(L, ctx, sr1, off1, sopts, False)   # same device index (raw reads)
        ns = min(n1, 20_000)
        hx = seed.SeedIndex(d.lr_seq, d.lr_off)
        want = hx.map(sr1[:off1[ns]], off1[:ns + 1], sopts, threads=min(16, os.cpu_count() or 1))
        hx.close()
        seed_check = {"reads": int(ns), "tasks": int(len(want)),
                      "equal": bool(np.array_equal(gpu_tasks[gpu_tasks["sr"] < ns], want))}
        if not seed_check["equal"]:
            raise SystemExit(f"bench: GPU seeding differs from the host path on the first {ns} reads")
        cpu, cpu_res = cpu_baseline(synth.with_seeds(dt, gpu_tasks), args.cpu_lrs_per_worker)
        del gpu_tasks
        parity = check_parity(it, cpu_res)
    if rank != 0:
        if cm is not None:
            cm.close()
        return
    value = total_bases * args.steps / el / 1e6 if not args.task_only else None
    step_ms = el / args.steps * 1e3 if not args.task_only else None
    task_ms = el_task / args.steps * 1e3
    dom_ms /= K
    dom_tops = dom_cells * OPS_PER_CELL / (dom_ms * 1e-3) / 1e12
    ext_ms /= K
    ext_tops = ext_cells * OPS_PER_CELL / (ext_ms * 1e-3) / 1e12 if ext_ms > 0 else 0.0
    sw_stage_ms /= K
    sw_cells /= K
    # pileup kernel: algorithmic bytes (SURVEY.md §8d model) / kernel time
    cns_bytes = sum_lseq + 4 * sum_ncig + 16 * n_aln + own_bases * (2 + 2 + 6 * 4 * 2)
    traffic = traffic_cns = traffic_ext = traffic_seed = None
    pmc_src = None
    prof = ROOT / PMC_FILE   # tools/pmc_summary.py of the rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    if prof.exists():
        try:
            pm = json.loads(prof.read_text())

            def hbm(prefix):
                return next((v.get("hbm_bytes_per_launch") for k, v in pm.items() if k.startswith(prefix)), None)
            traffic, traffic_cns = hbm("sw_global_pk_kernel<40"), hbm("cns_lr_kernel")
            ts = [hbm("prgpu::seed_batch_kernel"), hbm("prgpu::seed_wave_kernel")]   # both seeding passes
            ts = [hbm("seed_batch"), hbm("seed_wave")] if ts[0] is None else ts
            traffic_seed = sum(x for x in ts if x is not None) if ts[0] is not None else None
            traffic_ext = {k: v.get("hbm_bytes_per_launch") for k, v in pm.items() if k.startswith("sw_ext_")}
            pmc_src = f"{prof.name}: rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE passes per launch, " \
                      f"{pm.get('_build', 'build not recorded')}"
        except Exception:
            traffic = traffic_cns = traffic_ext = traffic_seed = None
    out = {
        "metric": "corrected long-read Mbases/sec per node",
        "value": round(value, 3) if value is not None else None,
        "unit": "Mbases/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 3) if step_ms is not None else None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic: iid genome, CLR-like long reads (15 % error), 50x 150 bp short reads in sequencer order, "
                "sampled per task by SeqChunker's chunk rule; the same dataset on every rank",
        "config": {
            "workload": "configs[1] per GPU: 4.6 Mb genome, 13,800 x 10 kb long reads (30x, 15% error), "
                        "50x 2x150 short reads; one whole sr-noccs correction run per step (read-long's output "
                        "restored in HBM, bwa-sr-1..N with mask_shortcut_frac, bwa-sr-finish)",
            "genome_bp": gl, "long_reads": n_lr, "long_read_bases": int(lr_off[-1]), "short_reads": n_sr,
            "owned_long_reads": hi - lo, "mode": mode,
            "parallelism": f"exact-parity layout x{world}: every rank indexes all {n_lr} long reads, seeds and aligns "
                           f"1/{world} of each task's short-read sample, alignments all-to-all to the long reads' "
                           f"owners over RCCL (pr_aln_exchange), corrected reads all-gathered (pr_lrset_commit)",
        },
        "loop": {"tasks": loop_rows, "device_ms": round(loop_dev_ms, 1), "chimera_lines": n_chim,
                 "same_task_list_every_step": same_tasks,
                 "repeat_identical": (first_digest == last_digest) if first_digest is not None else None,
                 "final_reads_sha256": last_digest},
        "value_task": round(total_bases / (task_ms * 1e-3) / 1e6, 3),
        "task": {"name": "bwa-sr-1", "ms": round(task_ms, 3), "short_reads": n1, "short_read_shard": s1 - s0,
                 "seeds": n_seeds, "alignments_received": int(n_recv), "coverage_cap": params1.coverage,
                 "wall_ms": task_wall},
        "stage_event_ms": {k: round(v, 3) for k, v in zip(("index", "seeding", "sw_extend", "sw_global_cigar",
                                                            "exchange_handoff", "consensus"), ev)},
        "sw_gcups": round(sw_cells / (sw_stage_ms * 1e-3) / 1e9, 2) if sw_stage_ms > 0 else None,
        "sw_gcups_note": "DP cells of every extension and CIGAR launch of the bwa-sr-1 task (unpruned band, SURVEY.md "
                         "§8d) / the SW stage's device time (HIP events: extension rounds incl. the bwa-mode walk and "
                         "final passes, then the CIGAR pass)",
        "sw_gcups_kernels": round((ext_cells + dom_cells) / ((ext_ms + dom_ms) * 1e-3) / 1e9, 2)
        if ext_ms + dom_ms > 0 else None,
        "bwa": {"rounds": bwa_rounds, "seeds_extended": bwa_ext, "patches": bwa_patch},
        "cigar_kernel_phase_share": {k: round(v / max(sum(pc), 1), 3) for k, v in
                                     zip(("masks", "dp", "backtrack", "emit"), pc)},
        "consensus_phase_ms_summed_over_workgroups": {k: round(v, 1) for k, v in cns_phases.items()},
        "seeding_phase_ms_summed_over_waves": seed_phases,
        "traffic_source": pmc_src,
        "roofline": {
            "kernel": "sw_global_pk_kernel<40> (ksw_global2 CIGAR pass + backtrack, packed int16, two tasks per lane)",
            "bound": "valu", "achieved": round(dom_tops, 3), "peak": round(VALU_PEAK_TOPS, 2), "unit": "TOP/s (int32)",
            "frac": round(dom_tops / VALU_PEAK_TOPS, 4), "traffic": traffic, "launch_ms": round(dom_ms, 3),
            "cells_per_launch": int(dom_cells), "ops_per_cell": OPS_PER_CELL,
            "peak_packed_int16": round(2 * VALU_PEAK_TOPS, 2),
            "frac_of_packed_int16_peak": round(dom_tops / (2 * VALU_PEAK_TOPS), 4),
        },
        "roofline_consensus": {
            "kernel": "cns_lr_kernel (bin cap + pileup + argmax, one long read per workgroup)", "bound": "hbm",
            "achieved": round(cns_bytes / (ev[5] * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(cns_bytes / (ev[5] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": int(cns_bytes),
            "alignments": int(n_aln), "traffic": traffic_cns, "launch_ms": round(ev[5], 3),
        },
        "roofline_extension": {
            "kernels": "every ksw_extend2 DP launch of the task (sw_ext_pk_kernel<40>, sw_ext_phase_kernel<*>, wide), "
                       "all bwa-mode rounds, both sides and band tries",
            "bound": "valu", "achieved": round(ext_tops, 3), "peak": round(VALU_PEAK_TOPS, 2), "unit": "TOP/s (int32)",
            "frac": round(ext_tops / VALU_PEAK_TOPS, 4), "summed_launch_ms": round(ext_ms, 3),
            "launches": ext_launches, "cells": int(ext_cells), "ops_per_cell": OPS_PER_CELL,
            "frac_of_packed_int16_peak": round(ext_tops / (2 * VALU_PEAK_TOPS), 4),
            "traffic_per_launch": traffic_ext,
        },
        "roofline_seeding": seeding_roofline(ev[1], s1 - s0, traffic_seed, n_seeds),
        "roofline_bwa_rounds": bwa_rounds_roofline(bwa_ms, n_seeds, bwa_ext, int(na_rep.value), bwa_rounds),
        "cpu_baseline": cpu,
        "cpu_baseline_reference": reference_cpu(),
        "comm": "rccl" if cm is not None else "none",
        "seed_parity_vs_host": seed_check,
        "gen_s": round(gen_s, 1),
        "upload_s": round(upload_s, 2),
        "reads_ok": ok,
        "parity": parity,
    }
    print(json.dumps(out), file=_JSON_OUT, flush=True)
    if cm is not None:
        cm.close()
    if parity is not None and parity["mismatches"]:
        raise SystemExit(f"bench: {parity['mismatches']} of {parity['checked_reads']} reads differ from the CPU chain")
    if first_digest is not None and first_digest != last_digest:
        raise SystemExit("bench: the correction run's output differs between steps")


def lrs_index_ms(L, ctx) -> float:
    from proovread_amd import seed
    return seed._last_ms(L.pr_seed_gpu_index_last_ms, ctx)


# Seeding's byte model (tools/seed_stats.py, the host build of the same core with work counters,
# on 20 k reads of this workload): per 150 bp read the scratch and index accesses the algorithm
# makes -- occurrence-table builds, SMEM steps, chaining and the filter -- in bytes.  Kept as a
# constant measured once ("seeding roofline").
# algorithmic bytes per short read of the seeding stage without its output (tools/seed_bytes.py on
# this dataset: 150 B of bases, 16 B per start's koff pair x 139.0 starts, 32 B per occurrence-table
# hit (kpos, kext, contig lookup) x 3200.5 hits), + 40 B per output seed (pr_seed_task)
SEED_BYTES_PER_READ = 104789
SEED_BYTES_PER_SEED = 40


def seeding_roofline(kernel_ms: float, n_reads: int, traffic, n_seeds: int = 0):
    if not SEED_BYTES_PER_READ or not kernel_ms:
        return {"kernel": "seed_batch_kernel + seed_wave_kernel", "bound": "hbm", "launch_ms": round(kernel_ms, 3),
                "traffic": traffic, "note": "byte model not measured"}
    alg = SEED_BYTES_PER_READ * n_reads + SEED_BYTES_PER_SEED * n_seeds
    ach = alg / (kernel_ms * 1e-3) / 1e9
    return {"kernel": "seed_batch_kernel + seed_wave_kernel", "bound": "hbm", "achieved": round(ach, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "alg_bytes": int(alg),
            "bytes_per_read": SEED_BYTES_PER_READ, "traffic": traffic, "launch_ms": round(kernel_ms, 3)}


# bwa mode's bookkeeping kernels (aln_walk_*_kernel, aln_final_*_kernel: mem_chain2aln's walk,
# mem_sort_dedup_patch .. mem_reg2sam) per task, in algorithmic bytes: every seed's task record
# read once by the walk (40 B, pr_seed_task's fields), every extended seed's result read by the
# walk and again by the final pass as a region (2 x 32 B: score, query / reference ends, true
# score, band, global score, flags), every reported alignment written once (32 B)
BWA_BYTES_PER_SEED, BWA_BYTES_PER_EXT, BWA_BYTES_PER_ALN = 40, 64, 32


def bwa_rounds_roofline(ms, n_seeds: int, n_ext: int, n_aln: int, rounds: int):
    walk, final, early = (float(x) for x in ms)
    alg = BWA_BYTES_PER_SEED * n_seeds + BWA_BYTES_PER_EXT * n_ext + BWA_BYTES_PER_ALN * n_aln
    t = walk + final + early
    ach = alg / (t * 1e-3) / 1e9 if t > 0 else 0.0
    return {"kernels": "aln_walk_wave_kernel / aln_walk_kernel (every round) + aln_final_wave_kernel / aln_final_kernel "
                       "(early pass on the side stream, complement and late passes on the main stream)",
            "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "alg_bytes": int(alg), "summed_launch_ms": round(t, 3),
            "walk_ms": round(walk, 3), "final_main_ms": round(final, 3), "final_early_side_ms": round(early, 3),
            "critical_path_ms": round(walk + final, 3), "rounds": rounds, "seeds": n_seeds, "extended": n_ext,
            "reported": n_aln}


if __name__ == "__main__":
    main()
