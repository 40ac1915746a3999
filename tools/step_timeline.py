"""One bench step's kernel timeline from a rocprofv3 kernel trace (the launches between the last
two mask_lr_kernel dispatches): start / duration / queue of every launch above a threshold."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.04
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "mask_lr_kernel" in r["Kernel_Name"]]
seg = rows[idx[-2] + 1:idx[-1] + 1]
t0 = int(seg[0]["Start_Timestamp"])
for r in seg:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("prgpu::", "")[:45]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    if d > thr:
        print(f"{s:8.2f} {d:7.3f} q{r['Queue_Id']} {n} grid={r['Grid_Size_X']}")
print("span ms", (int(seg[-1]["End_Timestamp"]) - t0) / 1e6)
