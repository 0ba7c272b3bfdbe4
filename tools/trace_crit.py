#!/usr/bin/env python3
"""Where the time of a block-Jacobi kernel trace goes (dev aid).

Splits the span of the last solve in a rocprofv3 --kernel-trace SQLite database
during which (a) an apply or Gram kernel is running (the chip is doing the
wide, GPU-filling work), (b) only EVD kernels run (one workgroup per pair:
the chip is mostly idle), (c) nothing of ours runs.  (b)+(c) is the latency
the two overlapped chains fail to hide.

    python tools/trace_crit.py run_results.db [more.db ...]
"""
import sqlite3
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def minus(a, b):
    """a \\ b for sorted disjoint interval lists."""
    out, j = [], 0
    for s, e in a:
        cur = s
        while j < len(b) and b[j][1] <= cur:
            j += 1
        k = j
        while k < len(b) and b[k][0] < e:
            if b[k][0] > cur:
                out.append([cur, b[k][0]])
            cur = max(cur, b[k][1])
            k += 1
        if cur < e:
            out.append([cur, e])
    return out


def kind(name):
    n = name.lower()
    if "svdj" not in n:
        return "torch"   # copies (simulated exchanges, copy-in), generator, norms
    if any(k in n for k in ("qbuild", "quad_update", "slab_reduce")):
        return "evd"  # the latency chain of a (quad) step: Q builds, Gram-space update
    for k in ("gram", "evd", "apply"):
        if k in n:
            return k
    return "other"


def main(path, last_solve=True):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    d = [dict(zip(cols, r)) for r in db.execute("select * from kernels")]
    d.sort(key=lambda x: x["start"])
    if last_solve:  # keep what follows the longest gap between kernels
        ends, mx = [], 0
        for x in d:
            mx = max(mx, x["end"])
            ends.append(mx)
        cut = max(range(1, len(d)), key=lambda i: d[i]["start"] - ends[i - 1])
        d = d[cut:]
    t0, t1 = d[0]["start"], max(x["end"] for x in d)
    by = defaultdict(list)
    for x in d:
        by[kind(x["name"])].append((x["start"], x["end"]))
    wide = union(by["gram"] + by["apply"] + by["other"] + by["torch"])
    evd = union(by["evd"])
    span = t1 - t0
    only_evd = length(minus(evd, wide))
    busy = length(union(wide + evd))
    gaps = sorted(minus([[t0, t1]], union(wide + evd)), key=lambda g: g[0] - g[1])
    print(f"{path}\n  {len(d)} kernels; span {span / 1e6:.2f} ms; wide (gram/apply) busy {length(wide) / 1e6:.2f} ms "
          f"({100 * length(wide) / span:.1f} %), EVD-only {only_evd / 1e6:.2f} ms "
          f"({100 * only_evd / span:.1f} %), idle {(span - busy) / 1e6:.2f} ms")
    for k, iv in sorted(by.items()):
        tot = sum(e - s for s, e in iv)
        print(f"  {k:6s} n={len(iv):6d} sum {tot / 1e6:9.2f} ms avg {tot / len(iv) / 1e3:8.1f} us "
              f"union {length(union(iv)) / 1e6:8.2f} ms")
    # launch-to-start delay per kernel kind: start minus the end of the
    # previous kernel on the same stream (dependency + dispatch latency)
    prev_end, delay = {}, defaultdict(list)
    for x in d:
        sid = x.get("stream_id", x.get("queue_id"))
        if sid in prev_end:
            delay[kind(x["name"])].append(max(0, x["start"] - prev_end[sid]) / 1e3)
        prev_end[sid] = x["end"]
    for k, v in sorted(delay.items()):
        v = sorted(v)
        print(f"  {k:6s} start delay after the stream's previous kernel: median {v[len(v) // 2]:.1f} us, "
              f"p90 {v[int(len(v) * 0.9)]:.1f} us, sum {sum(v) / 1e3:.2f} ms")
    hist = defaultdict(float)
    for s, e in gaps:
        us = (e - s) / 1e3
        hist[next(b for b in (5, 10, 20, 50, 100, 1e12) if us < b)] += us / 1e3
    print("  idle ms by gap length (us): " + ", ".join(
        f"<{b:g}: {v:.2f}" for b, v in sorted(hist.items())))
    big = sorted(gaps, key=lambda g: g[0] - g[1])[:6]
    for gs_, ge in big:
        before = max((x for x in d if x["end"] <= gs_), key=lambda x: x["end"])
        after = min((x for x in d if x["start"] >= ge), key=lambda x: x["start"])
        print(f"    gap {(ge - gs_) / 1e3:8.1f} us at {(gs_ - t0) / 1e6:8.2f} ms: after "
              f"{kind(before['name'])} -> before {kind(after['name'])} {after['name'][:50]}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
