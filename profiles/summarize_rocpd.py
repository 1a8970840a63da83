"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite) per kernel name."""
import sqlite3
import sys


def main(db, top=40, steps=None):
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                       "from kernels group by name order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"# {db}: {sum(r[1] for r in rows)} dispatches, total kernel time {tot/1e6:.3f} ms")
    if steps:
        print(f"# per step ({steps} steps profiled): {tot/1e6/steps:.3f} ms")
    print(f"{'pct':>7} {'calls':>7} {'avg_us':>9} {'min_us':>9} {'max_us':>9}  kernel")
    for r in rows[:top]:
        print(f"{r[2]/tot*100:6.2f}% {r[1]:7d} {r[3]/1e3:9.2f} {r[4]/1e3:9.2f} {r[5]/1e3:9.2f}  {r[0][:150]}")


if __name__ == "__main__":
    main(sys.argv[1], steps=int(sys.argv[2]) if len(sys.argv) > 2 else None)
