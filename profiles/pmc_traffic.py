"""Per-dispatch HBM bytes of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

FETCH_SIZE is doubled for gfx950 wide streaming reads (MI355X_MICROARCH.md, HBM section); WRITE_SIZE
is taken as reported.  Both are KB.  Grouped by grid size (one group per launch shape).
usage: python profiles/pmc_traffic.py FETCH_DB WRITE_DB KERNEL_SUBSTRING [OUT_JSON]
(OUT_JSON uses the schema bench.py's pmc_traffic() reads: kernels[<name without spaces>].mean_hbm_bytes_per_launch)
"""
import json
import sqlite3
import sys


def per_shape(db, kernel, counter):
    c = sqlite3.connect(db)
    rows = c.execute("select grid_size, count(*), avg(value) from counters_collection "
                     "where counter_name=? and kernel_name like ? group by grid_size",
                     (counter, f"%{kernel}%")).fetchall()
    return {g: (n, v) for g, n, v in rows}


def main(fetch_db, write_db, kernel, out_json=None):
    f = per_shape(fetch_db, kernel, "FETCH_SIZE")
    w = per_shape(write_db, kernel, "WRITE_SIZE")
    tot = []
    for g in sorted(f):
        fb = f[g][1] * 1024 * 2
        wb = w.get(g, (0, 0.0))[1] * 1024
        tot.append(fb + wb)
        print(f"grid {g}: {f[g][0]} dispatches  FETCH_SIZE {f[g][1]:.1f} KB (x2 = {fb/1e6:.2f} MB)  "
              f"WRITE_SIZE {w.get(g, (0, 0))[1]:.1f} KB  -> {(fb + wb)/1e6:.2f} MB/launch")
    if tot:
        print(f"mean over shapes: {sum(tot)/len(tot):.0f} B/launch")
    if out_json and tot:   # merged into an existing summary: one file can hold several kernels
        import os
        rec = json.load(open(out_json)) if os.path.exists(out_json) else {"kernels": {}}
        rec.setdefault("_method", "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, KB per "
                                  "dispatch; FETCH_SIZE doubled for gfx950 wide streaming reads (MI355X_MICROARCH.md "
                                  "HBM section), WRITE_SIZE as reported")
        rec["kernels"][kernel.replace(" ", "")] = {"mean_hbm_bytes_per_launch": round(sum(tot) / len(tot)),
                                                   "source": f"{fetch_db}, {write_db}"}
        json.dump(rec, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:5])
