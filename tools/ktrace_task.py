"""Print one task's kernel timeline from a rocprofv3 kernel-trace CSV (the window starting at the
N-th-from-last launch of a kernel whose name contains --anchor).

    python tools/ktrace_task.py run_kernel_trace.csv [--anchor seed_batch_kernel<false>] [--back 4] [--min-ms 0.15]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--anchor", default="seed_batch_kernel<false>")
ap.add_argument("--back", type=int, default=4)
ap.add_argument("--min-ms", type=float, default=0.15)
ap.add_argument("--n", type=int, default=400)
a = ap.parse_args()
r = sorted(csv.DictReader(open(a.csv)), key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if a.anchor in x["Kernel_Name"]]
i0 = idx[-a.back]
t0 = int(r[i0]["Start_Timestamp"])
for x in r[i0:i0 + a.n]:
    d = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
    if d >= a.min_ms:
        print(f"{(int(x['Start_Timestamp']) - t0) / 1e6:8.2f} {d:7.2f} q{x.get('Queue_Id', '')} {x['Kernel_Name'][:80]}")
