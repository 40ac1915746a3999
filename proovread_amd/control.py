"""Iteration control around the hot path (host side, bin/proovread):

  cov2seqchunker     short-read sampling per iteration (proovread:2085-2102): which
                     SeqChunker chunks feed the next bwa-proovread run;
  mask_shortcut      the skip rule on the masked fraction bpN/bpt (proovread:2026-2047);
  masked_fraction    bpN/bpt from the masking statistic (proovread:1711-1716; on the
                     GPU it is pr_iter_mask's device pair, all-reduced over ranks).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional


@dataclasses.dataclass
class Sampler:
    """The `$first_chunk` global of proovread (:546) and the cfg values it uses."""
    chunk_number: int = 1000   # proovread.cfg:195 sr-chunk-number
    chunk_step: int = 20       # proovread.cfg:196 sr-chunk-step
    first_chunk: int = 1
    sampling: bool = True      # --no-sampling turns it off

    def cov2seqchunker(self, c: float, tc: float) -> Optional[Dict[str, int]]:
        """SeqChunker parameters for sr coverage c and target tc, or None (no sampling)."""
        if not self.sampling:
            return None
        if c * 0.8 < tc:   # :2090 don't sample if the target is more than 80 % of the data
            return None
        per_step = int(self.chunk_step * (tc / c) + .5)
        sc = {"--chunk-number": self.chunk_number, "--chunk-step": self.chunk_step,
              "--chunks-per-step": per_step, "--first-chunk": self.first_chunk}
        self.first_chunk += per_step
        if self.first_chunk > self.chunk_step:
            self.first_chunk -= self.chunk_step
        return sc


def masked_fraction(bpt: int, bpn: int) -> float:
    return bpn / bpt   # proovread divides unguarded (:1716)


def mask_shortcut(tasks: List[str], tc: int, masked_frac: float, masked_fracs: List[float],
                  shortcut_frac: float = 0.92, min_gain: float = 0.03) -> str:
    """proovread:2026-2047 on the task list (edited in place like @TASKS).

    Returns "skip" (all but the last task dropped: masked > shortcut_frac, or the gain
    over the previous iteration < min_gain), "continue", or "" when the check does
    not apply (no shortcut fraction, or tc is the second-to-last task or later)."""
    if not shortcut_frac or tc >= len(tasks) - 2:
        return ""
    prev = masked_fracs[-1] if masked_fracs else -min_gain
    res = "continue"
    if masked_frac > shortcut_frac:
        res = "skip"
    elif prev and (masked_frac - min_gain) < prev:
        res = "skip"
    if res == "skip":
        del tasks[tc + 1:len(tasks) - 1]   # splice(@TASKS, $TC+1, $#TASKS-$TC-1)
    masked_fracs.append(masked_frac)
    return res
