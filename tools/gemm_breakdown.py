"""Per-launch-shape breakdown of gemm_kernel dispatches in a rocpd database (steps = profiled steps)."""
import collections
import sqlite3
import sys


def main(db, steps):
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, grid_y, grid_z, duration from kernels where name like '%gemm_kernel%'").fetchall()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, gx, gy, gz, d in rows:
        key = (n.split("<")[1].split(">")[0], gx // 256, gy, gz)
        agg[key][0] += 1
        agg[key][1] += d / 1e3
    tot = sum(v[1] for v in agg.values())
    for k, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(k, cnt, f"{t / steps:.1f} us/step", f"{t / cnt:.1f} us/call")
    print(f"gemm total per step {tot / steps / 1e3:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
