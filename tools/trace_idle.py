"""Device-idle windows in a rocprofv3 kernel trace (dev aid): every interval
longer than a threshold during which no kernel runs, with the kernels on
either side.

    python tools/trace_idle.py run_kernel_trace.csv [threshold_us] [show]
"""
from __future__ import annotations

import csv
import sys


def main(path: str, thr_us: float = 100.0, show: int = 4) -> None:
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60],
                   r["Stream_Id"]) for r in csv.DictReader(open(path)))
    first = next(i for i, r in enumerate(rows) if "svdj::" in r[2])
    t0 = rows[first][0]
    prev_end, prev = rows[first][1], rows[first]
    idle = []
    for i in range(first + 1, len(rows)):
        g = (rows[i][0] - prev_end) / 1e3
        if g > thr_us:
            idle.append((g, prev, rows[i]))
        if rows[i][1] > prev_end:
            prev_end, prev = rows[i][1], rows[i]
    span = (rows[-1][1] - t0) / 1e3
    print(f"span {span / 1e3:.2f} ms, idle windows > {thr_us:.0f} us: {len(idle)}, "
          f"total {sum(x[0] for x in idle) / 1e3:.2f} ms")
    for g, a, b in idle[:show]:
        print(f"  {g:9.1f} us idle at t={(a[1] - t0) / 1e3:10.1f} us")
        print(f"      after  [{a[3]}] {a[2]}")
        print(f"      before [{b[3]}] {b[2]}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 100.0,
         int(sys.argv[3]) if len(sys.argv) > 3 else 4)
