"""configs[0], one bwa-sr-1 iteration two ways on the GPU, compared read by read:

* file level, the way bin/proovread runs it (proovread:1254-1355, 1528-1621): the
  `bwa-proovread index` / `bwa-proovread mem -b BIN -l LEN <bwa-sr-1 options>` drop-ins
  (host seeding, pr_sw_run, SAM text, the -b/-l bin filter on the host), `samtools view
  -bS` and `samtools sort` (the BAM drop-ins), then `bam2cns --bam --ref` (BAM decode,
  pr_cns_run) writing the corrected .fq;
* in process: the loop's device stages (correct.GpuStages: the read set resident in HBM,
  index and seeding there, pr_iter_* = bwa-mode SW, the -b/-l filter on the device, hand-off in coordinate order,
  consensus) with no SAM/BAM in between.

Inputs: the bundled sample's long reads (read-long's output: the stubby filter, upper case)
and short reads simulated from the sample genome at 50x (the sample's short-read file is not
in the checkout).  The corrected sequences and qualities must be identical: the hand-off's
order, the device bin filter and the device seeding stand in for SAM order, the host filter
and the host seeding without changing a base."""
import io
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))

from proovread_amd import bam2cns, cns, correct, samtools  # noqa: E402
from proovread_amd import bwa_proovread as bp  # noqa: E402
from proovread_amd import tasks as T  # noqa: E402


def _read_fq(path):
    out = {}
    lines = Path(path).read_text().split("\n")
    for i in range(0, len(lines) - 3, 4):
        if lines[i].startswith("@"):
            out[lines[i][1:].split()[0]] = (lines[i + 1], lines[i + 3])
    return out


@pytest.mark.gpu
def test_file_level_chain_equals_device_iteration(tmp_path):
    from test_correct_loop import _sample_inputs
    _, lrs, srfq = _sample_inputs()
    reads, _ = correct.read_long(lrs, 300)   # stubby: 2 x the 150 bp short reads
    task, cov = "bwa-sr-1", 50.0
    tcov = T.sr_coverage(task)
    max_cov = min(cov, tcov) * 0.75                       # proovread:1540-1541
    bsz = T.bin_size("sr-noccs")
    blen = bsz * min(cov, tcov)                           # proovread:1302-1313
    lr_fq, lr_fa, sr_fq = tmp_path / "lr.fq", tmp_path / "lr.fa", tmp_path / "sr.fq"
    with open(lr_fq, "wb") as fq, open(lr_fa, "wb") as fa:
        for rid, s, q in zip(reads.ids, reads.seqs, reads.quals):
            fq.write(b"@%s\n%s\n+\n%s\n" % (rid.encode(), s, q))
            fa.write(b">%s\n%s\n" % (rid.encode(), s))
    sr_fq.write_bytes(srfq)

    # ---- file level: bwa-proovread -> samtools view -bS -> samtools sort -> bam2cns
    assert bp.index([str(lr_fa), str(lr_fa)], log=io.StringIO()) == 0
    sam = tmp_path / "x.sam"
    with open(sam, "w") as fh:
        rc = bp.mem(["-b", str(bsz), "-l", f"{blen:g}"] + T.bwa_argv(task) + [str(lr_fa), str(sr_fq)], out=fh,
                    log=io.StringIO())
    assert rc == 0
    ub, sb = tmp_path / "x.unsorted.bam", tmp_path / "x.bam"
    assert samtools.view(["-b", "-S", "-o", str(ub), str(sam)]) == 0
    assert samtools.sort(["-o", str(sb), str(ub)]) == 0
    pre = str(tmp_path / "cns")
    assert bam2cns.main(["--bam", str(sb), "--ref", str(lr_fq), "--prefix", pre, "--coverage", f"{max_cov:g}",
                         "--max-ins-length", "0", "--qv-offset", "33", "--append"]) == 0
    got_file = _read_fq(pre + ".fq")

    # ---- in process: the loop's device stages (the read set resident in HBM)
    names, seqs, _ = bp.read_fastx(str(sr_fq))
    sr, sr_off = bp._pool(seqs)
    st = correct.GpuStages()
    st.load(reads)
    params = cns.CnsParams(coverage=max_cov, use_ref_qual=True, detect_chimera=False, max_ins_length=0)
    st.task(task, sr, sr_off, params, (bsz, blen), mask_cfg=(correct.hcr_mask_for(task), 150))
    got = st.reads()
    out = [(0, s, q, []) for s, q in zip(got.seqs, got.quals)]   # pr_lrset_commit: every status 0

    assert len(got_file) > 0.9 * len(reads.ids)
    n_cmp = 0
    for rid, (status, s, q, _) in zip(reads.ids, out):
        if rid not in got_file:
            continue
        assert status == 0, rid
        fs, fq_ = got_file[rid]
        assert s.decode("latin-1") == fs, rid
        assert q.decode("latin-1") == fq_, rid
        n_cmp += 1
    assert n_cmp == len(got_file)
    # the iteration corrected the reads (not a pass-through comparison)
    raw = dict(zip(reads.ids, reads.seqs))
    changed = sum(got_file[r][0] != raw[r].decode("latin-1") for r in got_file)
    assert changed > 0.8 * len(got_file)
