#!/usr/bin/env python3
"""Kernel stats (the rocprofv3 --stats columns) from a rocprofv3 results .db (rocpd SQLite),
for runs made without --output-format csv.

  python scripts/db_kstats.py <results.db> <out.csv>
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = c.execute("select s.display_name, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.end - d.start) "
                     "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
                     "group by s.display_name").fetchall()
    total = sum(r[2] for r in rows) or 1
    rows.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, tot, mn, mx in rows:
            w.writerow([name, n, tot, tot / n, 100.0 * tot / total, mn, mx])
    for name, n, tot, mn, mx in rows[:20]:
        print("%-50s calls %5d avg_us %10.1f pct %5.1f" % (name[:50], n, tot / n / 1e3, 100.0 * tot / total))


if __name__ == "__main__":
    main()
