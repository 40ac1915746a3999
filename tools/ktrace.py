"""Per-kernel mean duration per step from a rocprofv3 kernel trace (ms), top N kernels."""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
pat = sys.argv[3] if len(sys.argv) > 3 else None
agg = defaultdict(lambda: [0, 0.0, 0.0])
for r in rows:
    n = r["Kernel_Name"].replace("void ", "").replace("prgpu::", "")[:60]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    a = agg[n]; a[0] += 1; a[1] += d; a[2] = max(a[2], d)
for n, (c, t, m) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    if pat and pat not in n: continue
    print(f"{t / steps:9.3f} ms/step  calls {c:5d}  max {m:8.3f}  {n}")
