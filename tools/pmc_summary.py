"""Per-kernel PMC summary of a rocprofv3 --pmc database (rocpd sqlite):
mean counter value per dispatch; FETCH_SIZE / WRITE_SIZE in bytes with FETCH_SIZE
doubled (gfx950 correction, MI355X_MICROARCH.md HBM section); SQ_* counters raw
(SQ_INSTS_* per wave instruction; SQ_*_CYCLES in quad-cycles)."""
import sqlite3
import sys


def main(db, out=None):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    rows = c.execute("select * from counters_collection").fetchall()
    idx = {k: i for i, k in enumerate(cols)}
    agg = {}
    for r in rows:
        name = r[idx["kernel_name"]].split("(")[0]
        cn = r[idx["counter_name"]]
        v = r[idx["value"]]
        d = agg.setdefault(name, {}).setdefault(cn, [])
        d.append(v)
    lines = ["%-32s %-20s %10s %16s %16s" % ("kernel", "counter", "dispatches", "mean/dispatch", "corrected")]
    for k, cs in sorted(agg.items()):
        for cn, vs in sorted(cs.items()):
            m = sum(vs) / len(vs)
            if cn in ("FETCH_SIZE", "WRITE_SIZE"):  # KiB -> bytes; FETCH_SIZE doubled (gfx950)
                corr = m * 1024 * (2 if cn == "FETCH_SIZE" else 1)
            else:
                corr = m
            lines.append("%-32s %-20s %10d %16.1f %16.0f" % (k[:32], cn, len(vs), m, corr))
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
