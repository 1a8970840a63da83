"""Per-kernel summary of a rocprofv3 rocpd database (results.db): name, calls, total/avg us, share;
optionally per (kernel, grid) with --grid.  Usage: python tools/dbstats.py run_results.db [--grid] [--top N]"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    by_grid = "--grid" in sys.argv
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, duration from kernels").fetchall()
    agg = collections.defaultdict(list)
    for n, g, d in rows:
        agg[(n, g) if by_grid else (n,)].append(d)
    tot = sum(sum(v) for v in agg.values())
    print(f"{'share':>7} {'calls':>6} {'total_us':>10} {'avg_us':>9}  kernel")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        name = k[0] if len(k[0]) < 110 else k[0][:107] + "..."
        extra = f" grid={k[1]}" if by_grid else ""
        print(f"{100 * sum(v) / tot:6.2f}% {len(v):6d} {sum(v) / 1e3:10.1f} {sum(v) / len(v) / 1e3:9.2f}  {name}{extra}")


if __name__ == "__main__":
    main()
