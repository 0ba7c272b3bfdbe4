"""Per-kernel effective clock from a rocprofv3 --kernel-trace --pmc run (dev aid).

    python tools/clock_summary.py <rocprofv3 -d directory>

Joins counter_collection.csv (GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES per
dispatch) with kernel_trace.csv (start/end) by dispatch id and prints, per
kernel name in dispatch order of first appearance, the median over its
dispatches of: wall us, clock GHz = GRBM_GUI_ACTIVE / 8 / wall, and MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clock x wall).
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main(d):
    ctr = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    trc = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not ctr or not trc:
        print("missing csv", ctr, trc)
        return
    wall = {}
    for r in csv.DictReader(open(trc[0])):
        wall[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(ctr[0])):
        did = r["Dispatch_Id"]
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    order, rows = [], collections.defaultdict(list)
    for did in sorted(per, key=lambda x: int(x)):
        k = names[did]
        if k not in rows:
            order.append(k)
        w = wall.get(did)
        if not w:
            continue
        c = per[did]
        clk = c["GRBM_GUI_ACTIVE"] / 8 / w
        mf = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * clk * w) if clk > 0 else 0.0
        rows[k].append((w * 1e6, clk / 1e9, mf))
    for k in order:
        v = rows[k]
        if not v:
            continue
        print("%-70s n=%3d  wall %8.1f us  clock %.3f GHz  MFMA busy %5.1f %%" % (
            k[:70], len(v), statistics.median(x[0] for x in v), statistics.median(x[1] for x in v),
            100 * statistics.median(x[2] for x in v)))


if __name__ == "__main__":
    main(sys.argv[1])
