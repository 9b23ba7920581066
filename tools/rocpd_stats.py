"""Per-kernel duration summary of a rocprofv3 rocpd database (the default output of
`rocprofv3 --kernel-trace --stats -d DIR -o run -- ...`), written in the column layout of
rocprofv3's own kernel_stats.csv.  Usage: python tools/rocpd_stats.py DB [OUT.csv]"""
import csv
import sqlite3
import sys


def main() -> None:
    db = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    con = sqlite3.connect(db)
    rows = con.execute(
        "select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start), "
        "avg((end-start)*(end-start)) from kernels group by name order by sum(end-start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"]
    recs = []
    for name, n, tot, avg, mn, mx, sq in rows:
        sd = max(sq - avg * avg, 0.0) ** 0.5
        recs.append([name, n, tot, f"{avg:.3f}", f"{100.0 * tot / total:.2f}", mn, mx, f"{sd:.3f}"])
    f = open(out, "w", newline="") if out else sys.stdout
    w = csv.writer(f, quoting=csv.QUOTE_ALL)
    w.writerow(hdr)
    w.writerows(recs)


if __name__ == "__main__":
    main()
