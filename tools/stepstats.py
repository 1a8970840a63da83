"""Per-step kernel time of a rocprofv3 kernel trace (rocpd db): steps delimited by a marker kernel
(default the fp32 ViT's patchify), averaged over steps [a, b).
usage: python tools/stepstats.py DB [--marker patchify_f32] [--steps 10 20] [--top 30]"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = sys.argv[sys.argv.index("--marker") + 1] if "--marker" in sys.argv else "patchify_f32"
    a, b = (int(x) for x in sys.argv[sys.argv.index("--steps") + 1:sys.argv.index("--steps") + 3]) \
        if "--steps" in sys.argv else (10, 20)
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    rows = sqlite3.connect(db).execute("select name, grid_x, duration, start from kernels order by start").fetchall()
    starts = [r[3] for r in rows if marker in r[0]]
    b = min(b, len(starts) - 1)
    lo, hi, ns = starts[a], starts[b], b - a
    agg, cnt = collections.defaultdict(float), collections.Counter()
    for n, g, d, st in rows:
        if lo <= st < hi:
            agg[(n[:80], g)] += d
            cnt[(n[:80], g)] += 1
    print(f"steps {a}..{b}: kernel time {sum(agg.values()) / ns / 1e3:.1f} us/step, span {(hi - lo) / ns / 1e3:.1f} us/step")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:top]:
        print(f"{v / ns / 1e3:8.1f} us/step {cnt[k] / ns:5.1f}/step  {k[0]} grid={k[1]}")


if __name__ == "__main__":
    main()
