"""Per-stream timeline of the block-step kernels from a rocprofv3 kernel trace
(dev aid for the latency-bound regime of many GPUs).

    python tools/trace_gaps.py gpurun_out/<dir>/run_kernel_trace.csv

For every (queue, stream) running svdj block kernels: kernel count, busy
time per kernel kind, the idle gaps between consecutive kernels, and the
span.  Also the whole-device union of busy intervals over the span of the
block kernels (how much of the wall time any kernel is running).
"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict


def kind(name: str) -> str | None:
    for k in ("gram_kernel", "evd_kernel", "apply_split_kernel", "apply_kernel"):
        if k in name:
            return k.replace("_kernel", "")
    return None


def main(path: str) -> None:
    rows = []
    for r in csv.DictReader(open(path)):
        k = kind(r["Kernel_Name"])
        if k is None:
            continue
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k,
                     (r["Queue_Id"], r["Stream_Id"])))
    rows.sort()
    if not rows:
        print("no block kernels")
        return
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    print(f"block kernels: {len(rows)}, span {(t1 - t0) / 1e6:.2f} ms")
    per = defaultdict(list)
    for r in rows:
        per[r[3]].append(r)
    for key, rs in sorted(per.items()):
        busy = defaultdict(float)
        cnt = defaultdict(int)
        gaps = []
        for i, (s, e, k, _) in enumerate(rs):
            busy[k] += (e - s) / 1e3
            cnt[k] += 1
            if i:
                gaps.append(max(s - rs[i - 1][1], 0) / 1e3)
        gaps.sort()
        tot = sum(gaps)
        med = gaps[len(gaps) // 2] if gaps else 0.0
        print(f"queue/stream {key}: {len(rs)} kernels, span {(rs[-1][1] - rs[0][0]) / 1e6:.2f} ms")
        for k in busy:
            print(f"   {k:12s} n={cnt[k]:6d} avg {busy[k] / cnt[k]:8.1f} us  total {busy[k] / 1e3:8.2f} ms")
        print(f"   gaps: total {tot / 1e3:.2f} ms, median {med:.1f} us, p90 "
              f"{gaps[int(len(gaps) * 0.9)] if gaps else 0:.1f} us")
    # union of busy intervals
    busy_u, cur_s, cur_e = 0, rows[0][0], rows[0][1]
    for s, e, _, _ in rows[1:]:
        if s > cur_e:
            busy_u += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy_u += cur_e - cur_s
    print(f"device busy (any block kernel running): {busy_u / (t1 - t0):.1%} of span")




def overlap(path: str) -> None:
    """Time during which >= 2 block kernels run at once, and which kinds."""
    ev = []
    for r in csv.DictReader(open(path)):
        k = kind(r["Kernel_Name"])
        if k:
            ev.append((int(r["Start_Timestamp"]), 1, k))
            ev.append((int(r["End_Timestamp"]), -1, k))
    ev.sort()
    running = defaultdict(int)
    last = ev[0][0]
    both = 0
    combo = defaultdict(float)
    for t, d, k in ev:
        n = sum(running.values())
        if n >= 2:
            both += t - last
            combo[tuple(sorted(x for x, c in running.items() for _ in range(c)))] += (t - last) / 1e6
        running[k] += d
        last = t
    print(f"two or more block kernels concurrently: {both / 1e6:.2f} ms")
    for c, v in sorted(combo.items(), key=lambda x: -x[1])[:6]:
        print(f"   {'+'.join(c):30s} {v:8.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
    overlap(sys.argv[1])
