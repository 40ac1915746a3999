"""Build libprgpu.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels
with the repository snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
SRC = PKG / "csrc"
OUT = PKG / "libprgpu.so"
SOURCES = ["cns_kernels.hip", "sw_kernels.hip", "pipe_kernels.hip", "mask_kernels.hip", "seed_kernels.hip",
           "sw_api.cpp", "prgpu_api.cpp", "seed.cpp", "trim.cpp", "bam_codec.cpp"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-pthread",
         # exact IEEE double semantics of the reference Perl arithmetic
         "-ffp-contract=off", "-fno-fast-math",
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def build(force: bool = False, verbose: bool = False) -> Path:
    srcs = [SRC / s for s in SOURCES if (SRC / s).exists()]
    deps = srcs + list(SRC.glob("*.h")) + [PKG.parent / "include" / "prgpu.h"]
    if not force and OUT.exists() and all(OUT.stat().st_mtime >= d.stat().st_mtime for d in deps):
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *FLAGS, "-o", str(OUT), *map(str, srcs), "-lz"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
