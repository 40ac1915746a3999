"""Summarise an SQ counter pass (tools/pmc_sq.sh) per kernel: wave cycles split into active /
waiting (s_waitcnt, barriers) / issue-stalled, VALU instructions per wave cycle, and the
VALU utilisation of the SIMDs (MI355X_MICROARCH.md: SQ cycle counters are quad-cycles).

    python tools/sq_summary.py gpurun_out/pmc_sq1 [out.json]
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
rows = list(csv.DictReader(open(d / "run_counter_collection.csv")))
agg = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("prgpu::", "")
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    calls[name].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
out = {}
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    wc = v.get("SQ_WAVE_CYCLES", 0.0)
    if wc <= 0:
        continue
    e = {"dispatches": len(calls[k]), "wave_cycles_q": wc}
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if c in v:
            e[c.replace("SQ_", "").lower() + "_frac"] = round(v[c] / wc, 3)
    if "SQ_INSTS_VALU" in v:
        e["valu_insts"] = v["SQ_INSTS_VALU"]
        e["valu_insts_per_wave_quadcycle"] = round(v["SQ_INSTS_VALU"] / wc, 3)
    if "SQ_INSTS_LDS" in v:
        e["lds_insts"] = v["SQ_INSTS_LDS"]
    if "SQ_WAVES" in v:
        e["waves"] = v["SQ_WAVES"]
    out[k] = e
txt = json.dumps(dict(list(out.items())[:25]), indent=1)
print(txt)
if len(sys.argv) > 2:
    Path(sys.argv[2]).write_text(txt + "\n")
