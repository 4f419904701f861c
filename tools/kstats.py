"""Summarise a rocprofv3 rocpd SQLite database: per-kernel calls / total / avg (us)."""
import sqlite3
import sys


def main(db, steps=None, top=40):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"{'calls':>7} {'total_us':>12} {'avg_us':>10} {'pct':>6}  kernel")
    for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{k:7d} {t:12.1f} {t / k:10.2f} {100 * t / tot:6.2f}  {n[:110]}")
    print(f"total kernel time {tot / 1e3:.2f} ms over {sum(v[0] for v in agg.values())} dispatches")


if __name__ == "__main__":
    main(sys.argv[1])
