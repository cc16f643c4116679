"""Kernel-duration summary (name, calls, avg/total us) from a rocprofv3 .db trace,
for runs made without --output-format csv."""
import csv
import sqlite3
import sys


def main(db, out=None):
    c = sqlite3.connect(db)
    q = ("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1000.0 from kernels "
         "group by name order by sum(end-start) desc")
    rows = [(n, k, round(a, 3), round(t, 3)) for n, k, a, t in c.execute(q)]
    tot = sum(r[3] for r in rows) or 1.0
    w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
    w.writerow(["Name", "Calls", "AverageUs", "TotalUs", "Percentage"])
    for r in rows:
        w.writerow(list(r) + [round(100 * r[3] / tot, 2)])


if __name__ == "__main__":
    main(*sys.argv[1:])
