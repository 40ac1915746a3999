"""`bwa-proovread mem` on its product path (bwa_proovread._mem_gpu: the seed index and the
seeds in HBM, bwa mode on them, the -b/-l filter on the device, SAM formatted natively by
pr_sw_sam) against the same CLI with the host seeding front end, the device SW and the
records formatted and binned in Python: byte-identical SAM, with and without -b/-l, FASTQ and
FASTA short reads, lowercase / N / IUPAC bases."""
import io

import numpy as np
import pytest

from proovread_amd import bwa_proovread as bp
from proovread_amd import sw

from test_bwa_proovread_cli import ARGS, _write


def _host_path(argv):
    out = io.StringIO()
    assert bp.mem(argv, out=out, sw_runner=lambda inp, wo: sw.run(inp, wo), log=io.StringIO()) == 0
    return out.getvalue()


def _gpu_path(argv):
    out = io.StringIO()
    log = io.StringIO()
    assert bp.mem(argv, out=out, log=log) == 0
    assert "(GPU)" in log.getvalue()
    return out.getvalue()


@pytest.mark.gpu
@pytest.mark.parametrize("binned", [True, False])
def test_gpu_mem_equals_host_seeding_path(tmp_path, binned):
    _write(tmp_path, np.random.default_rng(5))
    # reads the formatter must print as given: lowercase, N and an IUPAC code in a FASTQ read
    fq = (tmp_path / "sr.fq").read_text().split("\n")
    fq[1] = fq[1][:20].lower() + fq[1][20:40] + "N" + fq[1][41:60] + "R" + fq[1][61:]
    (tmp_path / "sr.fq").write_text("\n".join(fq))
    args = ARGS if binned else [x for i, x in enumerate(ARGS) if not (x in ("-b", "-l") or
                                                                     (i and ARGS[i - 1] in ("-b", "-l")))]
    argv = args + [str(tmp_path / "lr.fa"), str(tmp_path / "sr.fq")]
    want = _host_path(argv)
    got = _gpu_path(argv)
    assert got == want
    assert sum(1 for x in got.splitlines() if not x.startswith("@")) > 50


@pytest.mark.gpu
def test_gpu_mem_fasta_reads(tmp_path):
    _, srs = _write(tmp_path, np.random.default_rng(6))
    with open(tmp_path / "sr.fa", "w") as fh:
        for i, (r, _) in enumerate(srs):
            fh.write(f">sr{i}\n{r[:75]}\n{r[75:]}\n")
    argv = ARGS + [str(tmp_path / "lr.fa"), str(tmp_path / "sr.fa")]
    got = _gpu_path(argv)
    assert got == _host_path(argv)
    recs = [x.split("\t") for x in got.splitlines() if not x.startswith("@")]
    assert recs and all(r[10] == "*" for r in recs)
