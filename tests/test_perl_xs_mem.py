"""The Perl host boundary for the seed-extension stage: Prgpu::mem (perl/lib/Prgpu.pm over
the XS functions seed_index_build / seed_map / sw_run) produces what `bwa-proovread mem`
prints (bin/proovread:1313), i.e. proovread_amd/bwa_proovread.py:mem's SAM.

CPU: host seeding through XS gives the Python host's task list byte for byte, and with the
SW stage injected as the CPU oracle (as tests/test_bwa_proovread_cli.py does for the Python
CLI) the Perl records equal the Python records, with and without the -b/-l bin filter.
GPU: the same comparison with sw_run / pr_sw_run on the device on both sides.
"""
import io
import json
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from test_bwa_proovread_cli import ARGS, _write, oracle_runner
from proovread_amd import bwa_proovread as bp

ROOT = Path(__file__).resolve().parent.parent
HELPER = Path(__file__).resolve().parent / "perl_cns_helper.pl"
XS_SO = ROOT / "perl" / "lib" / "auto" / "Prgpu" / "Prgpu.so"

pytestmark = pytest.mark.skipif(shutil.which("perl") is None, reason="no perl")


@pytest.fixture(scope="module", autouse=True)
def xs_module():
    if not XS_SO.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "perl")], check=True)


def _inputs(tmp_path, args, odd_bases=False):
    _write(tmp_path, np.random.default_rng(5))
    if odd_bases:   # lowercase, N and IUPAC bases in some short reads (SEQ printing of both strands)
        lines = (tmp_path / "sr.fq").read_text().splitlines()
        for r, f in ((3, str.lower), (5, lambda x: x[:40] + "N" + x[41:]), (7, lambda x: x[:70] + "R" + x[71:]),
                     (11, lambda x: x[:20].lower() + x[20:100] + "NN" + x[102:])):
            lines[4 * r + 1] = f(lines[4 * r + 1])
        (tmp_path / "sr.fq").write_text("\n".join(lines) + "\n")
    argv = args + [str(tmp_path / "lr.fa"), str(tmp_path / "sr.fq")]
    a = bp.parse_mem(argv)
    so, wo = bp.options(a)
    lr_names, lr_seqs, _ = bp.read_fastx(a.ref)
    sr_names, sr_seqs, sr_quals = bp.read_fastx(a.reads)
    js = {
        "lr_names": lr_names, "lr_seqs": [s.decode() for s in lr_seqs],
        "sr_names": sr_names, "sr_seqs": [s.decode() for s in sr_seqs],
        "sr_quals": [q.decode() if q is not None else None for q in sr_quals],
        "seed_opts": {k: getattr(so, k) for k in ("min_seed_len", "min_chain_weight", "w", "split_factor",
                                                   "max_mem_intv", "max_occ", "drop_ratio", "a", "o_del",
                                                   "e_del", "o_ins", "e_ins")},
        "sw_opts": {k: getattr(wo, k) for k in ("a", "b", "o_del", "e_del", "o_ins", "e_ins", "w", "pen_clip5",
                                                 "pen_clip3", "zdrop", "min_score_per_base")},
        "b": a.b, "l": a.l, "threads": 2, "cl": " ".join(argv),
    }
    return argv, js


def _python_mem(argv, runner=None):
    out = io.StringIO()
    assert bp.mem(argv, out=out, sw_runner=runner, log=io.StringIO()) == 0
    lines = out.getvalue().splitlines(keepends=True)
    return [x for x in lines if x.startswith("@")], [x for x in lines if not x.startswith("@")]


def _perl_mem(js, tmp_path):
    p = tmp_path / "mem.json"
    p.write_text(json.dumps(js))
    r = subprocess.run(["perl", str(HELPER), "mem", str(p)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


@pytest.mark.parametrize("binning,odd", [(True, False), (False, False), (False, True)],
                         ids=["b20_l40", "no_filter", "odd_bases"])
def test_perl_mem_equals_python_mem_with_oracle_sw(tmp_path, binning, odd):
    # -l 40 (two reads' worth of bases per 20 bp bin) so the filter evicts on this small sample
    args = " ".join(ARGS).replace("-b 20 -l 225 ", "-b 20 -l 40 " if binning else "").split()
    argv, js = _inputs(tmp_path, args, odd)
    seen = {}
    oracle = oracle_runner("bwa-sr")

    def runner(inp, opts):
        seen["inp"] = inp
        seen["res"] = oracle(inp, opts)
        return seen["res"]

    head, rec = _python_mem(argv, runner)
    inp, res = seen["inp"], seen["res"]
    n = len(inp.t_sr)
    js["sw"] = {"pos": res["pos"].tolist(), "score": res["score"].tolist(), "pass": res["pass"].tolist(),
                "status": res["status"].tolist(), "cigar": [res.cigar_str(t) for t in range(res.n)],
                "task": res["task"].tolist(), "flag": res["flag"].tolist()}
    got = _perl_mem(js, tmp_path)
    # the task list Perl handed to the SW stage is the Python host's, byte for byte
    b = got["batch"]
    assert int(b["n_task"]) == n > 40
    for k, dt in (("t_sr", np.int32), ("t_lr", np.int32), ("t_strand", np.uint8), ("t_qbeg", np.int32),
                  ("t_rbeg", np.int32), ("t_slen", np.int32), ("t_chain", np.int32)):
        assert bytes.fromhex(b[k]) == np.asarray(getattr(inp, k[0:]), dt).tobytes(), k
    assert bytes.fromhex(b["sr_seq"]) == np.asarray(inp.sr_seq, np.uint8).tobytes()
    assert bytes.fromhex(b["lr_off"]) == np.asarray(inp.lr_off, np.int64).tobytes()
    assert got["head"] == head
    assert got["rec"] == rec
    if binning:
        assert len(rec) < sum(1 for t in range(res.n) if res["pass"][t])
    if odd:
        names = {x.split("\t")[0] for x in rec}
        assert {"sr3/1", "sr5/1", "sr11/1"} & names


@pytest.mark.gpu
def test_perl_mem_equals_python_mem_on_gpu(tmp_path):
    argv, js = _inputs(tmp_path, ARGS)
    head, rec = _python_mem(argv)
    got = _perl_mem(js, tmp_path)
    assert got["head"] == head
    assert got["rec"] == rec and len(rec) > 40


# ---- masking (SeqFilter --phred-mask) through XS

def _perl_mask(js, tmp_path):
    p = tmp_path / "mask.json"
    p.write_text(json.dumps(js))
    r = subprocess.run(["perl", str(HELPER), "mask", str(p)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


@pytest.mark.parametrize("spec,srl", [("20,41,80,130,60,0.7", 150), ("20,41,80,130,60,0.3", 101),
                                      ("15,40,75,125,30,0.5", 250)])
def test_perl_mask_params_equal_python(tmp_path, spec, srl):
    from proovread_amd import mask
    got = _perl_mask({"hcr_mask": spec, "min_sr_length": srl}, tmp_path)["params"]
    p = mask.params(spec, srl)
    for k in ("phred_min", "phred_max", "mask_min_len", "unmask_min_len", "mask_reduce", "phred_offset"):
        assert got[k] == getattr(p, k), k
    assert got["end_ratio"] == p.end_ratio


def test_perl_mask_without_device_dies(tmp_path):
    p = tmp_path / "mask.json"
    p.write_text(json.dumps({"hcr_mask": "20,41,80,130,60,0.7", "min_sr_length": 150, "seqs": ["ACGT"],
                             "quals": ["IIII"]}))
    r = subprocess.run(["perl", str(HELPER), "mask", str(p)], capture_output=True, text=True)
    assert r.returncode != 0 and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_perl_mask_equals_python_mask_on_gpu(tmp_path):
    import random
    from proovread_amd import mask
    rng = random.Random(9)
    seqs, quals = [], []
    for _ in range(40):
        L = rng.choice([0, 1, 64, 500, 3000, 10000])
        q, hi = [], rng.random() < 0.6
        while len(q) < L:
            q += [rng.randint(53, 74) if hi else rng.randint(33, 52)] * rng.randint(1, 400)
            hi = not hi
        quals.append(bytes(q[:L]).decode())
        seqs.append("".join(rng.choice("ACGT") for _ in range(L)))
    spec, srl = "20,41,80,130,60,0.7", 150
    got = _perl_mask({"hcr_mask": spec, "min_sr_length": srl, "seqs": seqs, "quals": quals}, tmp_path)
    want, wmcrs, wst = mask.run([s.encode() for s in seqs], [q.encode() for q in quals], mask.params(spec, srl))
    assert got["masked"] == [w.decode() for w in want]
    assert got["mcrs"] == wmcrs
    assert tuple(got["stats"]) == wst and wst[1] > 0


# ---- one iteration in one call (Prgpu::iteration -> iter_run -> pr_iter_*)

def _iter_inputs():
    from proovread_amd import synth
    d = synth.simulate(31, 60_000, 30, 3000, 40.0, sr_frac=0.3)
    asc = np.frombuffer(b"ACGTN", np.uint8)
    lr = [asc[d.lr_seq[d.lr_off[i]:d.lr_off[i + 1]]].tobytes().decode() for i in range(d.n_lr)]
    sr = [asc[d.sr_seq[d.sr_off[i]:d.sr_off[i + 1]]].tobytes().decode() for i in range(d.n_sr)]
    js = {"lr_ids": [f"lr{i}" for i in range(d.n_lr)], "lr_seqs": lr, "lr_quals": None, "sr_seqs": sr,
          "seed_opts": {"finish": 0}, "sw_opts": {"finish": 0}, "params": {"coverage": 11.25, "use_ref_qual": 1}}
    return d, js


def _perl_iter(js, tmp_path):
    p = tmp_path / "iter.json"
    p.write_text(json.dumps(js))
    r = subprocess.run(["perl", str(HELPER), "iter", str(p)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_perl_iteration_batch_equals_python_iteration_batch(tmp_path):
    """The batch Prgpu::iteration hands to iter_run: the host seeds in bwa mode (every seed of
    the kept chains, grouped by short read, with their chains) exactly as synth.with_seeds
    hands them to iteration.Iteration."""
    from proovread_amd import seed, synth
    d, js = _iter_inputs()
    js["inject"] = 1
    got = _perl_iter(js, tmp_path)
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    dd = synth.with_seeds(d, ix.map(d.sr_seq, d.sr_off, seed.default_opts(False), threads=2))
    b = got["batch"]
    assert int(b["n_task"]) == len(dd.t_sr) > 1000
    for k in ("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen", "t_chain"):
        assert bytes.fromhex(b[k]) == np.asarray(getattr(dd, k)).tobytes(), k
    assert "task_lr_off" not in b
    assert bytes.fromhex(b["lr_qual"]) == b"$" * int(d.lr_off[-1])
    assert bytes.fromhex(b["lr_seq"]) == np.asarray(d.lr_seq, np.uint8).tobytes()
    assert [r["status"] for r in got["res"]] == [-1] * d.n_lr


@pytest.mark.gpu
def test_perl_iteration_equals_python_iteration_on_gpu(tmp_path):
    from proovread_amd import cns, iteration, seed, sw, synth
    d, js = _iter_inputs()
    got = _perl_iter(js, tmp_path)["res"]
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    dd = synth.with_seeds(d, ix.map(d.sr_seq, d.sr_off, seed.default_opts(False), threads=2))
    it = iteration.Iteration(dd)
    it.launch(sw.default_opts(False), cns.CnsParams(coverage=11.25, use_ref_qual=True))
    want = it.results()
    assert len(got) == len(want) == d.n_lr
    for g, w in zip(got, want):
        assert g["status"] == w.status
        if w.status == 0:
            assert (g["seq"], g["qual"], g["trace"], g["cigar"]) == (w.seq, w.qual, w.trace, w.cigar_str)
            assert [tuple(c) for c in g["chim"]] == list(w.chim)
