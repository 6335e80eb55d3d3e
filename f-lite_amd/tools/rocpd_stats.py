"""Per-kernel summary (calls, total / average time, share) from a rocprofv3 rocpd SQLite database (its default
output when --output-format is not given). Usage: rocpd_stats.py run_results.db [--top N] [--grid]
(--grid splits rows by launch grid)."""
import argparse
import re
import sqlite3


def stats(db, by_grid=False):
    c = sqlite3.connect(db)
    agg = {}
    for name, dur, gx, gy, gz in c.execute("select name, duration, grid_x, grid_y, grid_z from kernels"):
        key = (re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", "")), (gx, gy, gz) if by_grid else None)
        n, t = agg.get(key, (0, 0))
        agg[key] = (n + 1, t + dur)
    total = sum(t for _, t in agg.values())
    return sorted(((k, n, t) for k, (n, t) in agg.items()), key=lambda r: -r[2]), total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--grid", action="store_true")
    a = ap.parse_args()
    res, total = stats(a.db, a.grid)
    print(f"total kernel time {total / 1e6:.3f} ms")
    for (name, grid), n, t in res[: a.top]:
        g = f" grid={grid}" if grid else ""
        print(f"{t / 1e6:10.3f} ms {100 * t / total:5.1f}% {n:6d} x {t / n / 1e3:9.1f} us  {name[:90]}{g}")


if __name__ == "__main__":
    main()
