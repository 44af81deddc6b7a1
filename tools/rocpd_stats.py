"""Per-kernel summary of a rocprofv3 --kernel-trace database (developer tool).

rocprofv3's default output is a rocpd SQLite database; this prints the same
columns as its `--stats` kernel_stats.csv (name, calls, total/avg/min/max ns,
percent) from the `kernels` view, so a database merged back from the GPU box
can be summarised here.

    python tools/rocpd_stats.py gpurun_out/prof13/run_results.db > profiles/r1_v13_kernel_stats.csv
"""
from __future__ import annotations

import csv
import sqlite3
import sys


def main() -> None:
    db = sqlite3.connect(sys.argv[1])
    rows = list(db.execute(
        "select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
        "from kernels group by name order by sum(end - start) desc"))
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, calls, tot, avg, mn, mx in rows:
        w.writerow([name, calls, tot, f"{avg:.1f}", f"{100.0 * tot / total:.2f}", mn, mx])


if __name__ == "__main__":
    main()
