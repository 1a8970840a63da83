"""Print one training step's kernel sequence (name, grid, duration, gap to previous end) from a
rocprofv3 --kernel-trace database.  A step is delimited by consecutive launches of a marker kernel."""
import sqlite3
import sys


def main(db, marker="zero_seed_kernel", which=-2):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels "
                       "order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    a, b = idx[which - 1], idx[which]
    # a side-stream kernel the step's graph starts just before the marker belongs to the step
    # (one kernel starting < 8 us before the marker)
    if a > 0 and rows[a][1] - rows[a - 1][1] < 8000 and marker not in rows[a - 1][0]:
        a -= 1
    if rows[b][1] - rows[b - 1][1] < 8000 and marker not in rows[b - 1][0] and b - 1 > a:
        b -= 1
    t0 = rows[a][1]
    tot = busy = 0
    prev_end = None
    print("#   dur_us  gap_us  start_us  (gap: start - previous kernel's end, in start order)")
    for r in rows[a:b]:
        d = (r[2] - r[1]) / 1e3
        gap = (r[1] - prev_end) / 1e3 if prev_end else 0.0
        prev_end = r[2]
        busy += d
        short = r[0].replace("void ", "").replace("pcv::", "")[:70]
        print(f"{d:8.2f} {gap:7.2f} {(r[1] - t0) / 1e3:8.2f}  grid=({r[3]},{r[4]},{r[5]})x{r[6]:<4d} {short}")
    span = (rows[b][1] - rows[a][1]) / 1e3
    print(f"# {b - a} kernels, busy {busy:.1f} us, span {span:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
