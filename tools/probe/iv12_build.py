"""Build the 12-byte SMEM-interval probe library:
seed_core.h with `Iv.occ` as uint32_t (12-byte intervals, iv_make narrowing the counts) and,
with --trace, a printf of every bwt_smem1a call's forward intervals and reported SMEMs (host and
device print the same lines, so a diff of the two names the first divergent step).  The product
sources are not touched: they are copied to a scratch tree and patched there.

    python tools/probe/iv12_build.py [--trace]  ->  tools/probe/libiv12[_trace].so
"""
import re
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
trace = "--trace" in sys.argv
tmp = Path("/tmp/iv12_probe")
shutil.rmtree(tmp, ignore_errors=True)
(tmp / "proovread_amd").mkdir(parents=True)
shutil.copytree(ROOT / "proovread_amd" / "csrc", tmp / "proovread_amd" / "csrc")
shutil.copytree(ROOT / "include", tmp / "include")
core = tmp / "proovread_amd" / "csrc" / "seed_core.h"
s = core.read_text()
s = s.replace("struct Iv {\n    int32_t start, end;\n    int64_t occ;\n};",
              "struct Iv {   // PROBE: 12 bytes\n    int32_t start, end;\n    uint32_t occ;\n};\n"
              "SC_HD Iv iv_make(int s, int e, int64_t o) { return Iv{s, e, (uint32_t)o}; }")
s = s.replace("static_assert(sizeof(Seed) == sizeof(Iv)", "static_assert(sizeof(Seed) >= sizeof(Iv)")
s = re.sub(r"\bIv (\w+)\{([^;]*)\};", r"Iv \1 = iv_make(\2);", s)
s = re.sub(r"= Iv\{([^;]*)\};", r"= iv_make(\1);", s)
if trace:
    s = s.replace("    const int ret = curr[nc - 1].end;   // the longest forward match\n",
                  "    const int ret = curr[nc - 1].end;   // the longest forward match\n"
                  "    printf(\"F x=%d min=%lld nc=%d\\n\", x, (long long)min_intv, nc);\n"
                  "    for (int j_ = 0; j_ < nc; ++j_) printf(\"  f %d %d %lld\\n\", curr[j_].start, curr[j_].end, (long long)curr[j_].occ);\n")
    s = s.replace("    iv_reverse(mem, nmem);\n    return ret;\n}",
                  "    iv_reverse(mem, nmem);\n"
                  "    printf(\"B x=%d nmem=%d\\n\", x, nmem);\n"
                  "    for (int j_ = 0; j_ < nmem; ++j_) printf(\"  m %d %d %lld\\n\", mem[j_].start, mem[j_].end, (long long)mem[j_].occ);\n"
                  "    return ret;\n}")
core.write_text(s)
flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-pthread", "-ffp-contract=off", "-fno-fast-math",
         "-Wno-unused-function", "-Wno-unused-variable", "-Wno-format"]
mine = ["seed_kernels.hip", "seed.cpp", "prgpu_api.cpp", "seed_index.hip"]
objs = []
for o in sorted((ROOT / "build" / "obj").glob("*.o")):
    src = o.name[:-2]
    if src in mine:
        out = tmp / (src + ".o")
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-c", "-o", str(out), str(tmp / "proovread_amd" / "csrc" / src)],
                       check=True)
        objs.append(str(out))
    else:
        objs.append(str(o))
lib = ROOT / "tools" / "probe" / ("libiv12_trace.so" if trace else "libiv12.so")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", "-o", str(lib), *objs,
                "-lz", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"], check=True)
print(lib)
