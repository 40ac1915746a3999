"""Device index over the F.antasticus long reads (ASCII, as the loop's long-read set holds them)
vs the host index: table digests, with the kext pass on the 4-bit and on the byte text."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_fantasticus_chain import FX  # noqa: E402

from proovread_amd import _abi, bwa_proovread as bp, seed  # noqa: E402

names, seqs, quals = bp.read_fastx(str(FX / "F.antasticus_long_error.fq"))
pool = np.frombuffer(b"".join(seqs), np.uint8).copy()
off = np.concatenate([[0], np.cumsum([len(s) for s in seqs])]).astype(np.int64)
ctx = _abi.default_context()
hx = seed.SeedIndex(pool, off)
names6 = ("text", "koff", "kpos", "kext", "cnt", "contigs")
for mode, v in (("nibble", "0"), ("nibble-loop", "2"), ("bytes", "1")):
    os.environ["PRGPU_INDEX_KEXT_BYTES"] = v
    dx = seed.DeviceSeedIndex(ctx, pool, off)
    a, b = dx.digest(), hx.digest()
    print(mode, "equal" if a == b else "DIFF", [n for n, x, y in zip(names6, a, b) if x != y])
