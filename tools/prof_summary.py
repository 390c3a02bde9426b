"""Summarise a rocprofv3 --kernel-trace --stats results database (rocpd sqlite)
into the per-kernel table committed under profiles/."""
import sqlite3
import sys


def main(db, out=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    lines = ["%-40s %8s %14s %12s %12s %12s %7s" % ("kernel", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "pct")]
    for name, n, s, a, lo, hi in rows:
        short = name.split("(")[0][:40]
        lines.append("%-40s %8d %14d %12.1f %12d %12d %6.2f%%" % (short, n, s, a, lo, hi, 100.0 * s / tot))
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
