"""proovread's per-task parameters (host side of the correction loop).

proovread.cfg is a Perl hash; bin/proovread looks values up with `cfg(KEY, TASK)`
(bin/proovread:1989-2024): a missing KEY loses a trailing `-<n>` (`bwa-mr-3` ->
`bwa-mr`), and in a per-task hash the TASK's own entry, else the TASK without its
counter, else DEF wins.  This module restates the entries the sr / mr correction loop
reads, with their cfg lines:

  mode-tasks      proovread.cfg:105-127 (sr-noccs, mr-noccs)
  bwa-*           proovread.cfg:318-365 (bwa mem options per task)
  sr-coverage     proovread.cfg:188-192
  hcr-mask        proovread.cfg:234-242
  bin-size        proovread.cfg:259-273 (bwa-proovread -b; -l = BIN x min(cov, task cov),
                  bin/proovread:1302-1313)

and the mode choice of bin/proovread:628-651 (`sr` up to 150 bp short reads, `mr`
beyond).  bwa mem options become pr_seed_opts / pr_sw_opts through the bwa-proovread
drop-in's own option parser, so a task's options mean exactly what `bwa-proovread mem`
would make of them.
"""
from __future__ import annotations

import re
from typing import Dict, List, Tuple

MODE_TASKS: Dict[str, Tuple[str, ...]] = {
    "sr-noccs": ("read-long", "bwa-sr-1", "bwa-sr-2", "bwa-sr-3", "bwa-sr-4", "bwa-sr-5", "bwa-sr-6", "bwa-sr-finish"),
    "mr-noccs": ("read-long", "bwa-mr-1", "bwa-mr-2", "bwa-mr-3", "bwa-mr-4", "bwa-mr-5", "bwa-mr-6", "bwa-mr-finish"),
}

# bwa mem option sets (proovread.cfg:318-365); '' = a bare flag
BWA_OPTS: Dict[str, List[str]] = {
    "bwa-sr": ["-a", "-Y", "-A", "5", "-B", "11", "-O", "2,1", "-E", "4,3", "-T", "2.5",
               "-k", "12", "-W", "20", "-w", "40", "-r", "1", "-D", "0", "-y", "20", "-L", "30,30"],
    "bwa-sr-finish": ["-a", "-Y", "-k", "17", "-W", "18", "-w", "30", "-r", "1.5", "-D", ".75", "-A", "5", "-B", "13",
                      "-O", "15,19", "-E", "3,3", "-T", "4", "-L", "30,30"],
    "bwa-mr-1": ["-a", "-Y", "-A", "5", "-B", "11", "-O", "2,1", "-E", "4,3", "-T", "2.5",
                 "-k", "12", "-W", "20", "-w", "40", "-r", "1", "-D", "0", "-y", "20", "-L", "30,30"],
    "bwa-mr": ["-a", "-Y", "-k", "13", "-W", "20", "-w", "40", "-r", "1", "-D", ".5", "-y", "20", "-A", "5", "-B", "11",
               "-O", "2,1", "-E", "4,3", "-T", "3", "-L", "30,30"],
    "bwa-mr-finish": ["-a", "-Y", "-k", "19", "-W", "40", "-w", "30", "-A", "5", "-B", "13", "-O", "15,19",
                      "-E", "3,3", "-T", "4", "-L", "30,30"],
}

SR_COVERAGE = {"DEF": 15.0, "bwa-sr-finish": 30.0, "bwa-mr-finish": 30.0}
HCR_MASK = {"DEF": "20,41,80,130,60,0.7", "bwa-mr-4": "20,41,80,130,60,0.3", "bwa-mr-5": "20,41,80,130,60,0.3",
            "bwa-mr-6": "20,41,80,130,60,0.3", "bwa-sr-4": "20,41,80,130,60,0.3", "bwa-sr-5": "20,41,80,130,60,0.3",
            "bwa-sr-6": "20,41,80,130,60,0.3"}
BIN_SIZE = {"DEF": 20, "sr": 20, "sr-noccs": 20, "mr": 50, "mr-noccs": 50}


def _strip(task: str) -> str:
    return re.sub(r"-\d+$", "", task)


def cfg_key(table: dict, key: str):
    """cfg(KEY) for a table of option sets: KEY, else KEY without its counter."""
    if key in table:
        return table[key]
    return table.get(_strip(key))


def cfg_task(table: dict, task: str):
    """cfg(KEY, TASK) of a per-task hash: the task, else the task without its counter, else DEF."""
    if task in table:
        return table[task]
    if _strip(task) in table:
        return table[_strip(task)]
    return table["DEF"]


def mode_for(min_sr_length: int) -> str:
    """bin/proovread:636-642: `mr` beyond 150 bp short reads (noccs: no PacBio subreads)."""
    return "mr-noccs" if min_sr_length > 150 else "sr-noccs"


def is_finish(task: str) -> bool:
    return task.endswith("-finish")


def bwa_argv(task: str) -> List[str]:
    opts = cfg_key(BWA_OPTS, task)
    if opts is None:
        raise ValueError(f"no bwa options for task {task}")
    return list(opts)


def options(task: str):
    """(pr_seed_opts, pr_sw_opts) of a bwa task, parsed as `bwa-proovread mem` parses them."""
    from . import bwa_proovread
    a = bwa_proovread.parse_mem(bwa_argv(task) + ["REF", "READS"])
    return bwa_proovread.options(a)


def sr_coverage(task: str) -> float:
    return float(cfg_task(SR_COVERAGE, task))


def hcr_mask(task: str) -> str:
    return cfg_task(HCR_MASK, task)


def bin_size(mode: str) -> int:
    return int(cfg_task(BIN_SIZE, mode))
