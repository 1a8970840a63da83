"""MFMA utilisation per kernel from rocprofv3 --pmc passes (tools/pmc_mfma.sh).

Pass "busy": SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE, GRBM_COUNT.
Pass "insts": SQ_INSTS_VALU_MFMA_MOPS_BF16 / _F32, SQ_INSTS_VALU_MFMA_BF16 / _F32, SQ_WAVE_CYCLES.

Per kernel (grouped by name and grid size):
  mfma_util = sum SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
              (rocprofv3's MfmaUtil expression, with GRBM_GUI_ACTIVE reported as the sum over the
              8 XCDs: MI355X_MICROARCH.md, DVFS give-back)
  mfma_tflops = SQ_INSTS_VALU_MFMA_MOPS_* x 512 FLOP / profiled duration
usage: python profiles/mfma_util.py BUSY_DB INSTS_DB [OUT_TXT] [--top N]
"""
import re
import sqlite3
import sys
from collections import defaultdict

SIMDS = 256 * 4
XCDS = 8


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*$", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:70]


def load(db):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, grid_size, counter_name, value, duration "
                     "from counters_collection").fetchall()
    per = defaultdict(dict)
    meta = {}
    for d, k, g, cn, v, dur in rows:
        per[d][cn] = per[d].get(cn, 0.0) + v
        meta[d] = (short(k), g, dur)
    return per, meta


def summarize(busy_db, insts_db):
    bper, bmeta = load(busy_db)
    iper, imeta = load(insts_db)
    agg = defaultdict(lambda: defaultdict(float))
    for per, meta in ((bper, bmeta), (iper, imeta)):
        for d, cnts in per.items():
            k = meta[d][:2]
            a = agg[k]
            tag = "b" if per is bper else "i"
            a["n_" + tag] += 1
            a["dur_" + tag] += meta[d][2]
            for cn, v in cnts.items():
                a[cn] += v
    out = []
    for (k, g), a in agg.items():
        nb, ni = max(a["n_b"], 1), max(a["n_i"], 1)
        gui = a["GRBM_GUI_ACTIVE"] / nb
        busy = a["SQ_VALU_MFMA_BUSY_CYCLES"] / nb
        util = busy / (gui / XCDS * SIMDS) if gui > 0 else 0.0
        mops = (a["SQ_INSTS_VALU_MFMA_MOPS_BF16"] + a["SQ_INSTS_VALU_MFMA_MOPS_F32"]) / ni
        dur_i = a["dur_i"] / ni
        tf = mops * 512 / (dur_i * 1e-9) / 1e12 if dur_i > 0 else 0.0
        out.append(dict(kernel=k, grid=g, n=int(a["n_b"]), dur_us=a["dur_b"] / nb / 1e3, tot_us=a["dur_b"] / 1e3,
                        util=util, tflops=tf, mops_bf16=a["SQ_INSTS_VALU_MFMA_MOPS_BF16"] / ni,
                        mops_f32=a["SQ_INSTS_VALU_MFMA_MOPS_F32"] / ni))
    out.sort(key=lambda r: -r["tot_us"])
    return out


def main(argv):
    top = 25
    if "--top" in argv:
        i = argv.index("--top")
        top = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    rows = summarize(argv[0], argv[1])
    lines = [f"{'kernel':70s} {'grid':>9s} {'n':>5s} {'avg_us':>8s} {'tot_us':>9s} {'mfma_util':>9s} {'TF/s':>7s}"]
    tot = sum(r["tot_us"] for r in rows)
    wutil = sum(r["util"] * r["tot_us"] for r in rows) / tot if tot else 0.0
    for r in rows[:top]:
        lines.append(f"{r['kernel']:70s} {r['grid']:9d} {r['n']:5d} {r['dur_us']:8.2f} {r['tot_us']:9.1f} "
                     f"{100 * r['util']:8.1f}% {r['tflops']:7.1f}")
    lines.append(f"time-weighted MFMA utilisation over all profiled kernels: {100 * wutil:.1f}%")
    txt = "\n".join(lines)
    print(txt)
    if len(argv) > 2:
        open(argv[2], "w").write(__doc__.split("usage")[0] + "\nsource dbs: " + argv[0] + ", " + argv[1] + "\n\n" + txt + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
