"""Kernel statistics (name, calls, total / average / min / max ns, share) from a rocprofv3
database (rocpd sqlite, the default output format) or a kernel_stats.csv: the summary
committed under profiles/."""
import csv
import glob
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    return rows


def main(argv):
    src, out = argv[0], argv[1]
    dbs = glob.glob(src + "/**/*.db", recursive=True) if not src.endswith(".db") else [src]
    rows = from_db(dbs[0])
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
        for n, k, s, a, mn, mx in rows:
            w.writerow([n, k, s, round(a, 1), mn, mx, round(100.0 * s / tot, 3)])
    for n, k, s, a, *_ in rows[:12]:
        print(f"{100.0 * s / tot:6.2f}%  {k:5d}  avg {a / 1e6:9.3f} ms  {n[:110]}")


if __name__ == "__main__":
    main(sys.argv[1:])
