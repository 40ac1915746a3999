"""The Perl host boundary: XS binding of libprgpu's consensus stage (perl/Prgpu.xs,
perl/lib/Prgpu.pm, perl/bin/prgpu-cns).

CPU: the module loads and reports the library version; without a device it dies
loudly (no fallback); the XS layer rejects buffers shorter than the batch's counts;
the Perl-side packing of every golden case is byte-identical to the Python host's
pr_cns_batch (proovread_amd/cns.py:pack_chunk).
GPU: a Perl process runs the golden cases through XS -> pr_cns_run and reproduces the
reference Perl engine's expected FASTQ / chimera lines (tests/golden/cns_expected.txt);
the prgpu-cns driver writes the same .fq / .chim.tsv as the bam2cns drop-in.
"""
import json
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import casefmt
from cns_case_util import case_inputs, params_key

ROOT = Path(__file__).resolve().parent.parent
HELPER = Path(__file__).resolve().parent / "perl_cns_helper.pl"
GOLD = Path(__file__).resolve().parent / "golden"
CASES = casefmt.read_cases(GOLD / "cns_cases.txt")
EXPECT = casefmt.read_expect(GOLD / "cns_expected.txt")
XS_SO = ROOT / "perl" / "lib" / "auto" / "Prgpu" / "Prgpu.so"

pytestmark = pytest.mark.skipif(shutil.which("perl") is None, reason="no perl")


@pytest.fixture(scope="module", autouse=True)
def xs_module():
    if not XS_SO.exists():   # build() makes it; a fresh checkout gets it here (gcc, ~1 s)
        subprocess.run(["make", "-s", "-C", str(ROOT / "perl")], check=True)
    return XS_SO


def _perl(*args, check=True):
    return subprocess.run(["perl", "-I", str(ROOT / "perl" / "lib"), *args], capture_output=True, text=True,
                          check=check)


def _chunk_json(items, params, path):
    reads, alns = [], []
    for c, lr, _ in items:
        reads.append({"id": lr.id, "seq": lr.seq, "qual": lr.qual, "desc": lr.desc, "length": lr.len})
        alns.append(list(c.sam))
    p = {"coverage": params.coverage, "max_ins_length": params.max_ins_length,
         "use_ref_qual": int(params.use_ref_qual), "detect_chimera": int(params.detect_chimera),
         "qual_weighted": int(params.qual_weighted)}
    path.write_text(json.dumps({"reads": reads, "alns": alns, "params": p}))
    return path


def _groups(include_noref=True):
    groups = {}
    for c in CASES:
        lr, alns, params = case_inputs(c)
        if params.qual_weighted or (c.p("noref") == "1" and not include_noref):
            continue
        key = params_key(params) + (c.p("noref") == "1",)
        groups.setdefault(key, (params, []))[1].append((c, lr, alns))
    return list(groups.values())


def test_module_loads_and_reports_version():
    from proovread_amd import _abi
    r = _perl("-MPrgpu", "-e", "print Prgpu::version()")
    assert r.stdout == _abi.lib().pr_version().decode()


def test_no_device_dies_loudly():
    r = _perl("-MPrgpu", "-e", "Prgpu::Context->new(0)", check=False)
    assert r.returncode != 0
    assert "pr_ctx_create" in r.stderr and "no HIP device" in r.stderr


def test_xs_rejects_short_buffers():
    code = ("my $b = Prgpu::pack_chunk([{id=>'r', seq=>'ACGT', qual=>'!!!!'}],"
            " [[qq{q\\t0\\tr\\t1\\t60\\t4M\\t*\\t0\\t0\\tACGT\\tIIII\\tAS:i:20}]]);"
            " substr($b->{aln_pos}, 2) = ''; Prgpu::cns_run(0, {}, $b)")
    r = _perl("-MPrgpu", "-e", code, check=False)
    assert r.returncode != 0
    assert "batch field 'aln_pos' holds 2 bytes, 4 needed" in r.stderr


def test_xs_null_context_is_an_argument_error():
    code = "Prgpu::run_chunk(0, {}, [{id=>'r', seq=>'ACGT', qual=>'!!!!'}], [[]])"
    r = _perl("-MPrgpu", "-e", code, check=False)
    assert r.returncode != 0 and "pr_cns_run: null ctx" in r.stderr


def test_prgpu_cns_driver_without_device_exits_255(tmp_path):
    (tmp_path / "ref.fq").write_text("@r\nACGT\n+\n!!!!\n")
    (tmp_path / "alns.sam").write_text("")
    r = _perl(str(ROOT / "perl" / "bin" / "prgpu-cns"), "--ref", str(tmp_path / "ref.fq"), "--sam",
              str(tmp_path / "alns.sam"), "--prefix", str(tmp_path / "xs"), check=False)
    assert r.returncode == 255 and "no HIP device" in r.stderr
    assert not (tmp_path / "xs.fq").exists()


@pytest.mark.parametrize("gi", range(len(_groups())))
def test_perl_packing_equals_python_packing(gi, tmp_path):
    """Every golden chunk packed by Prgpu.pm is byte-identical to cns.pack_chunk."""
    from proovread_amd import cns
    params, items = _groups()[gi]
    js = _chunk_json(items, params, tmp_path / "chunk.json")
    got = json.loads(_perl(str(HELPER), "pack", str(js)).stdout)
    d = cns.pack_chunk([x[1] for x in items], [x[2] for x in items])
    assert int(got["n_lr"]) == len(items)
    pool_len = {"seq_pool": int(d["_seq_pool_len"][0]), "qual_pool": int(d["_seq_pool_len"][0]),
                "cig_pool": 4 * int(d["_cig_pool_len"][0])}
    want_keys = {k for k in d if not k.startswith("_")}
    assert set(got) - {"n_lr"} == want_keys
    for k in want_keys:
        b = np.ascontiguousarray(d[k]).tobytes()
        if k in pool_len:
            b = b[:pool_len[k]]
        assert bytes.fromhex(got[k]) == b, k


@pytest.mark.gpu
def test_perl_xs_gpu_matches_reference(tmp_path):
    """A Perl process calls pr_cns_run through XS on every golden chunk."""
    n = 0
    for gi, (params, items) in enumerate(_groups()):
        js = _chunk_json(items, params, tmp_path / f"chunk{gi}.json")
        res = json.loads(_perl(str(HELPER), "run", str(js)).stdout)
        assert len(res) == len(items)
        for (c, _, _), r in zip(items, res):
            e = EXPECT[c.name]
            if e.error:
                assert r["status"] != 0, c.name
                continue
            assert r["status"] == 0, (c.name, r["status"])
            assert r["fastq"].rstrip("\n").split("\n") == e.fastq, c.name
            assert r["trace"] == e.trace, c.name
            assert [l.rstrip("\n") for l in r["chim_lines"]] == e.chim, c.name
            n += 1
    assert n >= 40


@pytest.mark.gpu
def test_prgpu_cns_driver_matches_bam2cns_dropin(tmp_path):
    """perl/bin/prgpu-cns (a Perl host over XS) writes the reference engine's FASTQ for a chunk."""
    params, items = max(((p, [x for x in it if not EXPECT[x[0].name].error])
                         for p, it in _groups(include_noref=False)), key=lambda g: len(g[1]))
    # distinct read ids so the chunk is one FASTQ and one SAM file
    fq, sam = [], []
    for k, (c, lr, _) in enumerate(items):
        rid = f"lr{k}"
        fq.append(f"@{rid} {lr.desc}".rstrip() + f"\n{lr.seq}\n+\n{lr.qual}\n")
        for l in c.sam:
            f = l.split("\t")
            f[2] = rid
            sam.append("\t".join(f).rstrip("\n") + "\n")
    (tmp_path / "ref.fq").write_text("".join(fq))
    (tmp_path / "alns.sam").write_text("".join(sam))
    flags = ["--coverage", str(params.coverage), "--max-ins-length", str(params.max_ins_length)]
    if not params.use_ref_qual:
        flags.append("--no-use-ref-qual")
    if params.detect_chimera:
        flags.append("--detect-chimera")
    r = _perl(str(ROOT / "perl" / "bin" / "prgpu-cns"), "--ref", str(tmp_path / "ref.fq"), "--sam",
              str(tmp_path / "alns.sam"), "--prefix", str(tmp_path / "xs"), *flags, check=False)
    assert r.returncode == 0, r.stderr
    got_fq = (tmp_path / "xs.fq").read_text()
    want = []
    for k, (c, _, _) in enumerate(items):
        e = EXPECT[c.name]
        want.append("\n".join([f"@lr{k}"] + e.fastq[1:]) + "\n")
    assert got_fq == "".join(want)
