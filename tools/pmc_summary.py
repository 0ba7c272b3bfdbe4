#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh) per kernel.

Reads every ``*counter_collection.csv`` under OUTDIR (one row per dispatch and
counter), sums each counter over a kernel's dispatches, and prints a markdown
table of derived rates:

* MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (dispatch time * 2.4 GHz * 1024 SIMDs); the counter
  is per-SIMD cycles (64 per v_mfma_f32_32x32x2_f32, checked against SQ_INSTS_MFMA), so
  this is the fraction of the fp32 MFMA peak at the 2.4 GHz peak clock.  GRBM_GUI_ACTIVE
  sums over the 8 XCDs and is not used as the clock
* issue mix  = SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_ANY over SQ_WAVE_CYCLES
* LDS bank conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
* HBM bytes  = FETCH_SIZE (x2, the gfx950 wide-stream under-count), WRITE_SIZE; GB/s over
  the summed dispatch time of the pass that measured them
* L2 hit     = TCC_HIT / (TCC_HIT + TCC_MISS)

Usage: python tools/pmc_summary.py OUTDIR
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import re
import sys

SIMDS = 1024  # 256 CUs x 4 SIMDs on MI355X
CLOCK = 2.4e9  # peak shader clock (Hz)


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    name = name.split("(")[0]
    name = name.replace("svdj::", "")
    return name[:60]


def load(outdir):
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    gui = collections.defaultdict(float)  # (pass, kernel) -> GRBM_GUI_ACTIVE
    where = {}  # counter -> pass that measured it
    ndisp = collections.defaultdict(set)
    dur = collections.defaultdict(lambda: collections.defaultdict(dict))  # ctr-set -> kernel -> disp -> ns
    for path in sorted(glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"),
                                 recursive=True)):
        tag = os.path.relpath(path, outdir).split(os.sep)[0]
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row.get("Kernel_Name", "?"))
                c = row.get("Counter_Name", "?")
                v = float(row.get("Counter_Value", 0) or 0)
                d = (tag, row.get("Dispatch_Id", row.get("Correlation_Id", "")))
                if c == "GRBM_GUI_ACTIVE":
                    gui[(tag, k)] += v
                else:
                    sums[k][c] += v
                    where[c] = tag
                ndisp[k].add(d)
                s, e = row.get("Start_Timestamp"), row.get("End_Timestamp")
                if s and e:
                    dur[tag][k][d] = int(e) - int(s)
    return sums, ndisp, dur, gui, where


def main():
    outdir = sys.argv[1]
    sums, ndisp, dur, gui_by, where = load(outdir)

    def pass_time(k, counter):
        # summed dispatch time (s) of the pass that measured `counter`
        tag = where.get(counter)
        return sum(dur.get(tag, {}).get(k, {}).values()) / 1e9 if tag else 0.0

    def pct(a, b):
        return f"{100.0 * a / b:.1f} %" if b else "-"

    print("| kernel | dispatches | MFMA busy | active / wait-inst / wait-any | LDS bank conflict |"
          " HBM read GB/s (x2) | HBM write GB/s | L2 hit |")
    print("|---|---|---|---|---|---|---|---|")
    order = sorted(sums, key=lambda k: -pass_time(k, "SQ_WAVE_CYCLES"))
    for k in order[:12]:
        s = sums[k]
        cyc = pass_time(k, "SQ_VALU_MFMA_BUSY_CYCLES") * CLOCK
        wc = s.get("SQ_WAVE_CYCLES", 0)
        mix = "-"
        if wc:
            mix = " / ".join(pct(s.get(x, 0), wc) for x in
                             ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"))
        tr = pass_time(k, "FETCH_SIZE")
        tw = pass_time(k, "WRITE_SIZE")
        rd = f"{2 * s['FETCH_SIZE'] * 1024 / tr / 1e9:.0f}" if tr and "FETCH_SIZE" in s else "-"
        wr = f"{s['WRITE_SIZE'] * 1024 / tw / 1e9:.0f}" if tw and "WRITE_SIZE" in s else "-"
        hit, miss = s.get("TCC_HIT_sum", 0), s.get("TCC_MISS_sum", 0)
        print(f"| {k} | {len(ndisp[k]) // max(1, len(dur))} | "
              f"{pct(s.get('SQ_VALU_MFMA_BUSY_CYCLES', 0), cyc * SIMDS) if 'SQ_VALU_MFMA_BUSY_CYCLES' in s else '-'} | "
              f"{mix} | {pct(s.get('SQ_LDS_BANK_CONFLICT', 0), s.get('SQ_LDS_IDX_ACTIVE', 0))} | "
              f"{rd} | {wr} | {pct(hit, hit + miss)} |")
    print()
    print("Raw counter sums per kernel:")
    print()
    for k in order[:6]:
        t = pass_time(k, "SQ_WAVE_CYCLES")
        print(f"* `{k}` ({t * 1e3:.1f} ms in pass 1): "
              + ", ".join(f"{c}={v:.4g}" for c, v in sorted(sums[k].items())))


if __name__ == "__main__":
    main()
