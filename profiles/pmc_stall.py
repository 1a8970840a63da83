"""Per-kernel issue / stall breakdown from tools/pmc_stall.sh (rocprofv3 --pmc passes).

Per kernel (grouped by name and grid): average duration, per-wave instruction counts (VALU, MFMA,
LDS, SALU, SMEM, VMEM), and the share of wave-cycles spent issuing (ACTIVE_INST_ANY), parked in
s_waitcnt / barriers (WAIT_ANY) and stalled on issue (WAIT_INST_ANY).
usage: python profiles/pmc_stall.py WAITS_DB INSTS_DB [--top N]"""
import sys
from collections import defaultdict

from mfma_util import load


def main(argv):
    top = 20
    if "--top" in argv:
        i = argv.index("--top")
        top = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    agg = defaultdict(lambda: defaultdict(float))
    for db in argv[:2]:
        per, meta = load(db)
        for d, cnts in per.items():
            k = meta[d][:2]
            a = agg[k]
            a["n_" + db] += 1
            a["dur_" + db] += meta[d][2]
            for cn, v in cnts.items():
                a[cn] += v
    rows = []
    for (k, g), a in agg.items():
        nw, ni = max(a["n_" + argv[0]], 1), max(a["n_" + argv[1]], 1)
        waves = a["SQ_WAVES"] / nw
        wc = a["SQ_WAVE_CYCLES"]
        pw = lambda c: a[c] / ni / max(waves, 1)  # noqa: E731  (per wave, from the insts pass)
        rows.append((a["dur_" + argv[0]] / nw / 1e3 * nw, k, g, a["dur_" + argv[0]] / nw / 1e3, waves,
                     pw("SQ_INSTS_VALU"), pw("SQ_INSTS_VALU_MFMA_BF16") + pw("SQ_INSTS_VALU_MFMA_F32"), pw("SQ_INSTS_LDS"),
                     pw("SQ_INSTS_SALU"), pw("SQ_INSTS_VMEM"), a["SQ_LDS_BANK_CONFLICT"] / ni,
                     a["SQ_ACTIVE_INST_ANY"] / max(wc, 1), a["SQ_WAIT_ANY"] / max(wc, 1),
                     a["SQ_WAIT_INST_ANY"] / max(wc, 1), a["SQ_ACTIVE_INST_VALU"] / max(wc, 1),
                     a["SQ_ACTIVE_INST_LDS"] / max(wc, 1)))
    rows.sort(key=lambda r: -r[0])
    print(f"{'kernel':60s} {'grid':>8s} {'avg_us':>7s} {'waves':>7s} {'valu/w':>7s} {'mfma/w':>7s} {'lds/w':>7s} "
          f"{'salu/w':>7s} {'vmem/w':>7s} {'bankcf':>9s} {'issue%':>6s} {'wait%':>6s} {'stall%':>6s} {'valu%':>6s} {'lds%':>6s}")
    for r in rows[:top]:
        print(f"{r[1][:60]:60s} {r[2]:8d} {r[3]:7.2f} {r[4]:7.0f} {r[5]:7.0f} {r[6]:7.0f} {r[7]:7.0f} {r[8]:7.0f} "
              f"{r[9]:7.0f} {r[10]:9.0f} {100*r[11]:6.1f} {100*r[12]:6.1f} {100*r[13]:6.1f} {100*r[14]:6.1f} {100*r[15]:6.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
