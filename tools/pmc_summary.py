"""Summarise the PMC passes of tools/pmc.sh into profiles/<name>.json.

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch.  On gfx950
FETCH_SIZE counts 64 B per 128-B line fetched, for every access width and pattern
calibrated on MI355X (16 / 4 / 1 B per lane, one dword per line, hashed lines:
tools/fetch_calib.hip -> profiles/r03_fetch_calibration.json), so the read figure is
doubled to the bytes of the lines moved; WRITE_SIZE reads the written bytes exactly.
"""
import csv
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

root = Path(__file__).resolve().parents[1]
out = Path(sys.argv[1]) if len(sys.argv) > 1 else root / "profiles" / "pmc_r01.json"
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = root / "gpurun_out" / f"pmc_{c}" / "run_counter_collection.csv"
    agg = defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    vals[c] = agg
res = {}
for name in vals["WRITE_SIZE"]:
    short = name.split("(")[0].replace("void ", "").replace("prgpu::", "")
    fe = vals["FETCH_SIZE"].get(name, [0.0])
    wr = vals["WRITE_SIZE"][name]
    fe_b = sum(fe) / len(fe) * 1024
    wr_b = sum(wr) / len(wr) * 1024
    if fe_b + wr_b < 1e6:
        continue
    res[short] = {
        "dispatches": len(wr),
        "fetch_bytes_per_launch_raw": round(fe_b),
        "fetch_bytes_per_launch_x2": round(2 * fe_b),
        "write_bytes_per_launch": round(wr_b),
        "hbm_bytes_per_launch": round(2 * fe_b + wr_b),
    }
res["_note"] = __doc__.strip()
res["_build"] = "build " + os.environ.get("PMC_BUILD", "not recorded")
out.write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res, indent=1))
