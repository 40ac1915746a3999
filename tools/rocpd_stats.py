"""Kernel statistics from a rocprofv3 rocpd database (the --kernel-trace output written as
SQLite by ROCm 7): per kernel name, calls, total / average / min / max duration (ns), as the
--stats CSV lists them.  python tools/rocpd_stats.py RUN_results.db [OUT.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                     f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    return rows


def main(argv):
    rows = stats(argv[0])
    tot = sum(r[2] for r in rows) or 1
    out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage")]
    out += [(r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(100.0 * r[2] / tot, 3)) for r in rows]
    if len(argv) > 1:
        with open(argv[1], "w", newline="") as f:
            csv.writer(f).writerows(out)
    for r in out[:40]:
        print(*(str(x)[:70] for x in r), sep="\t")
    return 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1:]))
