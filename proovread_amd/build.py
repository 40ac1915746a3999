"""Build libprgpu.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels
with the repository snapshot to the GPU box).  Sources compile to objects in
parallel (one hipcc per file, rebuilt when the file or any header changed), then
one link."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
SRC = PKG / "csrc"
OBJ = PKG.parent / "build" / "obj"
OUT = PKG / "libprgpu.so"
SOURCES = ["cns_kernels.hip", "sw_kernels.hip", "pipe_kernels.hip", "xchg_kernels.hip", "mask_kernels.hip", "seed_kernels.hip", "seed_index.hip", "aln_kernels.hip",
           "sw_api.cpp", "prgpu_api.cpp", "comm.cpp", "seed.cpp", "trim.cpp", "bam_codec.cpp", "fastq.cpp"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-pthread",
         # exact IEEE double semantics of the reference Perl arithmetic
         "-ffp-contract=off", "-fno-fast-math",
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
LIBS = ["-lz", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def _hipcc() -> str:
    return os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def build(force: bool = False, verbose: bool = False) -> Path:
    srcs = [SRC / s for s in SOURCES if (SRC / s).exists()]
    headers = list(SRC.glob("*.h")) + [PKG.parent / "include" / "prgpu.h"]
    hdr_t = max(h.stat().st_mtime for h in headers)
    OBJ.mkdir(parents=True, exist_ok=True)

    def obj_of(s: Path) -> Path:
        return OBJ / (s.name + ".o")

    def stale(s: Path) -> bool:
        o = obj_of(s)
        return force or not o.exists() or o.stat().st_mtime < max(s.stat().st_mtime, hdr_t)

    todo = [s for s in srcs if stale(s)]

    def compile_one(s: Path) -> None:
        cmd = [_hipcc(), *FLAGS, "-c", "-o", str(obj_of(s)), str(s)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)

    if todo:
        with ThreadPoolExecutor(max_workers=min(len(todo), os.cpu_count() or 4, 16)) as ex:
            list(ex.map(compile_one, todo))
    objs = [obj_of(s) for s in srcs]
    if force or todo or not OUT.exists() or any(OUT.stat().st_mtime < o.stat().st_mtime for o in objs):
        cmd = [_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", "-o", str(OUT), *map(str, objs), *LIBS]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    # the synthetic-workload generator of the bench and the scale tests (host C, not product)
    syn_src, syn_out = SRC / "synth.c", PKG / "libprsynth.so"
    if force or not syn_out.exists() or syn_out.stat().st_mtime < syn_src.stat().st_mtime:
        cmd = ["gcc", "-O3", "-fPIC", "-shared", "-pthread", "-std=c11", "-Wall", "-o", str(syn_out), str(syn_src)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
