"""Multi-rank consensus fan-out (proovread_amd/cns_shard.py), the drop-in for
`cat TASK.cmds | xargs -P N bam2cns` (bin/proovread:1596-1637).

CPU: command-file parsing, round-robin chunk dealing, and a real world_size-2
gloo run (chunks without --ref: bam2cns processes no read, bam2cns:313-320, so
no GPU is needed) checking every chunk's files are written exactly once.
GPU: all chunks of a golden command file, dealt to 2 ranks, merged in byfile
order, equal the per-read reference outputs.
"""
import functools
import os
import socket
from pathlib import Path

import pytest

import bamio
from proovread_amd import bam2cns, cns_shard


def test_round_robin_dealing():
    assert cns_shard.my_chunks(7, 0, 3) == [0, 3, 6]
    assert cns_shard.my_chunks(7, 2, 3) == [2, 5]
    got = sorted(i for r in range(4) for i in cns_shard.my_chunks(10, r, 4))
    assert got == list(range(10))


def test_read_cmds_param_join_format(tmp_path):
    # param_join (bin/proovread:1945) writes sorted "--key value" / "--flag" tokens
    f = tmp_path / "t.cmds"
    f.write_text("--append 1 --bam x.bam --bin-size 20 --coverage 15 --detect-chimera --prefix p.0\n\n"
                 "--append 1 --bam x.bam --prefix p.1\n")
    cmds = cns_shard.read_cmds(str(f))
    assert len(cmds) == 2 and cmds[0][-1] == "p.0"
    a = bam2cns.parse_args(cmds[0])
    assert a.append and a.detect_chimera and a.coverage == "15" and a.bam == "x.bam"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, cmds_file):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    assert cns_shard.main([cmds_file]) == 0


def test_gloo_two_ranks_write_every_chunk(tmp_path):
    bamio.write_bam(str(tmp_path / "x.bam"), [("r1", 100)], [])
    n = 5
    lines = [f"--append 1 --bam {tmp_path}/x.bam --max-ref-seqs 100 --prefix {tmp_path}/t.{i}"
             for i in range(n)]
    cmds = tmp_path / "t.cmds"
    cmds.write_text("\n".join(lines) + "\n")
    import torch.multiprocessing as mp
    mp.start_processes(_rank_main, args=(2, _free_port(), str(cmds)), nprocs=2, join=True,
                       start_method="spawn")
    for i in range(n):
        for ext in (".fq", ".chim.tsv", ".ignored.tsv"):
            assert (tmp_path / f"t.{i}{ext}").exists()


@pytest.mark.gpu
def test_two_rank_dealing_matches_reference(tmp_path):
    import test_bam2cns_cli as T
    p, cases = T._golden_group()
    fq = T._write_inputs(tmp_path, cases)
    offs, o = [], 0
    for c in cases:
        offs.append(o)
        o += len("\n".join(c.ref)) + 1
    base = f"--append 1 --sam {tmp_path}/x.sam --ref {fq} --max-ref-seqs 1 " + " ".join(T._cli_args(p))
    cmds = [(base + f" --ref-offset {off} --prefix {tmp_path}/t.{i}").split() for i, off in enumerate(offs)]
    assert cns_shard.run(cmds, 0, 2) == list(range(0, len(cases), 2))
    assert cns_shard.run(cmds, 1, 2) == list(range(1, len(cases), 2))
    files = sorted((str(x) for x in tmp_path.glob("t.[0-9]*.fq")), key=functools.cmp_to_key(bam2cns.byfile_cmp))
    merged = "".join(Path(f).read_text() for f in files).rstrip("\n").split("\n")
    want = [l for c in cases for l in T.EXPECT[c.name].fastq]
    assert merged == want
