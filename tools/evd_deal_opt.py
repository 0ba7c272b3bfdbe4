#!/usr/bin/env python3
"""LDS bank-conflict model and optimiser for the EVD kernel's block dealing.

The LDS EVD (csrc/hip/block.hip, evd_kernel) gives every thread up to
MAXOFF off-diagonal slot-pair blocks (a < b) for the whole kernel
(EvdDeal).  Every step a thread reads the 4 G entries of each block at
static position-space addresses, reads the two slots' rotation records and
writes the 4 moved entries.  Which block goes to which thread is free except
for the W "duty" blocks (wave 0, lanes 0..W-1, j = 0), so the assignment can
be chosen to keep the 32 lanes of every LDS lane group on distinct banks.

This tool
  * models the LDS cycles of one step for a dealing (ds_read_b32 /
    ds_write_b32: two 32-lane groups, bank = dword mod 32; the 8-byte record
    reads: two 32-lane groups, bank = dword mod 64, equal addresses
    broadcast) -- the conflict share of the round-2 dealing comes out close
    to the PMC SQ_LDS_BANK_CONFLICT share (profiles/r2_evd_unroll);
  * builds a dealing greedily, 32-lane group by group, picking the block
    that adds the fewest conflict cycles;
  * writes csrc/hip/evd_deal_tables.hpp (constexpr tables used for fp32 by
    EvdDeal; the kernel's static_assert re-checks them).

    python tools/evd_deal_opt.py            # report + write the header
    python tools/evd_deal_opt.py --check    # report only
"""
from __future__ import annotations

import argparse
import os

NT = 1024
CYC, BIP = 0, 1


class Ord:
    def __init__(self, W, order):
        self.W, self.o = W, order

    def pos_next(self, P):
        W = self.W
        if self.o == CYC:
            return P if P == 2 * W - 1 else (0 if P + 1 == 2 * W - 1 else P + 1)
        return P if P < W else (2 * W - 1 if P == W else P - 1)

    def prev_pos(self, P):
        W = self.W
        if self.o == CYC:
            return P if P == 2 * W - 1 else (2 * W - 2 if P == 0 else P - 1)
        return P if P < W else (W if P == 2 * W - 1 else P + 1)

    def slot_of(self, pos):
        W = self.W
        if self.o == CYC:
            return 0 if pos == 2 * W - 1 else (pos + 1 if pos <= W - 2 else 2 * W - 2 - pos)
        return pos if pos < W else pos - W

    def next_meeting(self, P1, P2):
        W = self.W
        if self.o == CYC:
            R = 2 * W - 1
            if P1 == R or P2 == R:
                o = P2 if P1 == R else P1
                if self.pos_next(o) != R - 1:
                    return -1
                return 1 if P1 == R else 0
            n1, n2 = self.pos_next(P1), self.pos_next(P2)
            if self.slot_of(n1) != self.slot_of(n2):
                return -1
            return 2 * self.slot_of(n1) + (1 if n1 <= W - 2 else 0)
        n1, n2 = self.pos_next(P1), self.pos_next(P2)
        if (n1 < W) == (n2 < W) or self.slot_of(n1) != self.slot_of(n2):
            return -1
        return 2 * self.slot_of(n1) + (1 if n1 < W else 0)

    def first_pos(self, a):
        return (2 * self.W - 1 if a == 0 else a - 1) if self.o == CYC else a

    def second_pos(self, a):
        return 2 * self.W - 2 - a if self.o == CYC else self.W + a


def tri_idx(N, i, j):
    a, b = min(i, j), max(i, j)
    return a * N - a * (a + 1) // 2 + (b - a - 1)


def block_duty(O, a, b):
    for e in range(4):
        x = O.second_pos(a) if e >> 1 else O.first_pos(a)
        y = O.second_pos(b) if e & 1 else O.first_pos(b)
        mt = O.next_meeting(x, y)
        if mt >= 0:
            return 256 * e + mt
    return -1


def round2_deal(W, order):
    """The dealing of EvdDeal (round 2): duty blocks first, then rows in
    complementary pairs 0, W-2, 1, W-3, ..."""
    O = Ord(W, order)
    duty = []
    for s in range(W):
        a = O.slot_of(O.prev_pos(O.first_pos(s)))
        b = O.slot_of(O.prev_pos(O.second_pos(s)))
        duty.append((min(a, b), max(a, b)))
    rest = []
    for i in range(W - 1):
        a = W - 2 - (i >> 1) if i & 1 else i >> 1
        for b in range(a + 1, W):
            if block_duty(O, a, b) < 0:
                rest.append((a, b))
    return duty, rest


def block_addrs(W, order, a, b, esize=4):
    """(4 read dwords, 4 write dwords, 2 record slots) of block (a, b)."""
    O = Ord(W, order)
    N = 2 * W
    pa, pb = (O.first_pos(a), O.second_pos(a)), (O.first_pos(b), O.second_pos(b))
    rd, wr = [], []
    for e in range(4):
        x, y = pa[e >> 1], pb[e & 1]
        rd.append(tri_idx(N, x, y) * esize // 4)
        wr.append(tri_idx(N, O.pos_next(x), O.pos_next(y)) * esize // 4)
    return rd, wr, (a, b)


def group_cost(addrs_per_instr, nbanks_list):
    """LDS cycles of one 32-lane group: per instruction max over banks of the
    number of distinct addresses."""
    tot = 0
    for addrs, nb in zip(addrs_per_instr, nbanks_list):
        banks = {}
        for ad in addrs:
            banks.setdefault(ad % nb, set()).add(ad)
        tot += max((len(s) for s in banks.values()), default=1)
    return tot


def deal_cost(W, order, slots):
    """slots[j][tid] = (a, b) or None.  Returns (cycles, conflict-free cycles)
    of one step's G reads, G writes and record reads (per the tables in
    MI355X_MICROARCH.md section LDS)."""
    cyc = ideal = 0
    for j in range(len(slots)):
        for g0 in range(0, NT, 32):
            blks = [slots[j][t] for t in range(g0, g0 + 32) if slots[j][t] is not None]
            if not blks:
                continue
            info = [block_addrs(W, order, a, b) for a, b in blks]
            instr = [[x[0][e] for x in info] for e in range(4)]
            instr += [[x[1][e] for x in info] for e in range(4)]
            # 8-byte records: slot s at dwords 2s, 2s+1, bank = dword mod 64,
            # so slots conflict when equal mod 32 (and differ)
            instr += [[x[2][0] for x in info], [x[2][1] for x in info]]
            c = group_cost(instr, [32] * 10)
            cyc += c
            ideal += 10
    return cyc, ideal


def slots_from(duty, rest, W):
    maxoff = (W * (W - 1) // 2 + NT - 1) // NT
    flat = list(duty) + list(rest)
    flat += [None] * (maxoff * NT - len(flat))
    return [[flat[j * NT + t] for t in range(NT)] for j in range(maxoff)]


def optimise(W, order, seed_rest):
    """Greedy: fill the non-duty slots 32-lane group by group; each lane takes
    the remaining block adding the fewest conflict cycles to its group."""
    duty, _ = round2_deal(W, order)
    maxoff = (W * (W - 1) // 2 + NT - 1) // NT
    total = len(duty) + len(seed_rest)
    # slot positions g (flat index) that hold non-duty blocks, in g order
    free = [g for g in range(len(duty), total)]
    info = {blk: block_addrs(W, order, *blk) for blk in seed_rest}
    remaining = list(seed_rest)
    flat = list(duty) + [None] * (maxoff * NT - len(duty))
    # groups: flat index g -> (j, tid), group id (j, tid // 32)
    by_group = {}
    for g in free:
        j, t = divmod(g, NT)
        by_group.setdefault((j, t // 32), []).append(g)
    for key in sorted(by_group):
        gs = by_group[key]
        used = [dict() for _ in range(10)]   # instr -> bank -> set(addr)
        j, grp = key
        # blocks already in this group (duty blocks of wave 0, j = 0)
        for t in range(grp * 32, grp * 32 + 32):
            g = j * NT + t
            if g < len(duty):
                rd, wr, (a, b) = block_addrs(W, order, *duty[g])
                for i, ad in enumerate(rd + wr + [a, b]):
                    used[i].setdefault(ad % 32, set()).add(ad)
        for g in gs:
            best, bestc = None, None
            for idx, blk in enumerate(remaining):
                rd, wr, (a, b) = info[blk]
                c = 0
                for i, ad in enumerate(rd + wr + [a, b]):
                    s = used[i].get(ad % 32)
                    if s and ad not in s:
                        c += len(s)
                if bestc is None or c < bestc:
                    best, bestc = idx, c
                    if c == 0:
                        break
            blk = remaining.pop(best)
            flat[g] = blk
            rd, wr, (a, b) = info[blk]
            for i, ad in enumerate(rd + wr + [a, b]):
                used[i].setdefault(ad % 32, set()).add(ad)
    return [[flat[j * NT + t] for t in range(NT)] for j in range(maxoff)]


def local_search(W, order, slots, ndut, iters=60000, seed=1):
    """Random pairwise swaps of non-duty blocks between lane groups, kept when
    the two groups' modelled cycles drop."""
    import random
    rng = random.Random(seed)
    maxoff = len(slots)
    info = {}

    def addrs(blk):
        if blk not in info:
            info[blk] = block_addrs(W, order, *blk)
        return info[blk]

    def gcost(j, grp):
        blks = [slots[j][t] for t in range(grp * 32, grp * 32 + 32) if slots[j][t] is not None]
        if not blks:
            return 0
        inf = [addrs(b) for b in blks]
        instr = [[x[0][e] for x in inf] for e in range(4)] + [[x[1][e] for x in inf] for e in range(4)]
        instr += [[x[2][0] for x in inf], [x[2][1] for x in inf]]
        return group_cost(instr, [32] * 10)

    free = [(j, t) for j in range(maxoff) for t in range(NT)
            if slots[j][t] is not None and j * NT + t >= ndut]
    for _ in range(iters):
        (j1, t1), (j2, t2) = rng.sample(free, 2)
        g1, g2 = (j1, t1 // 32), (j2, t2 // 32)
        if g1 == g2:
            continue
        before = gcost(*g1) + gcost(*g2)
        slots[j1][t1], slots[j2][t2] = slots[j2][t2], slots[j1][t1]
        if gcost(*g1) + gcost(*g2) > before:
            slots[j1][t1], slots[j2][t2] = slots[j2][t2], slots[j1][t1]
    return slots


def header(tables):
    out = ["// Generated by tools/evd_deal_opt.py -- do not edit.",
           "// Bank-conflict-optimised block dealing of the fp32 EVD (EvdDeal): entry",
           "// j * 1024 + tid = (a << 8) | b of thread tid's j-th slot-pair block, 0xffff",
           "// if none; the first W entries are the duty blocks (checked by",
           "// evd_deal_ok in block.hip).",
           "#pragma once", "", "namespace svdj {", ""]
    for (W, order), slots in tables.items():
        name = f"kEvdDealF32_W{W}_{'bip' if order == BIP else 'cyc'}"
        vals = []
        for j in range(len(slots)):
            for t in range(NT):
                blk = slots[j][t]
                vals.append(0xffff if blk is None else (blk[0] << 8) | blk[1])
        out.append(f"constexpr unsigned short {name}[{len(vals)}] = {{")
        for i in range(0, len(vals), 16):
            out.append("    " + ", ".join(f"0x{v:04x}" for v in vals[i:i + 16]) + ",")
        out.append("};")
        out.append("")
    out.append("}  // namespace svdj")
    return "\n".join(out) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--iters", type=int, default=60000, help="local-search swaps per table")
    args = ap.parse_args()
    tables = {}
    for W, order in ((64, BIP), (64, CYC), (32, BIP), (32, CYC)):
        duty, rest = round2_deal(W, order)
        s0 = slots_from(duty, rest, W)
        c0, i0 = deal_cost(W, order, s0)
        s1 = optimise(W, order, rest)
        s1 = local_search(W, order, s1, len(duty), iters=args.iters)
        c1, i1 = deal_cost(W, order, s1)
        print(f"W={W} {'bip' if order == BIP else 'cyc'}: round-2 dealing {c0} LDS cycles/step "
              f"({100 * (c0 - i0) / c0:.1f} % conflicts), optimised {c1} ({100 * (c1 - i1) / c1:.1f} %)",
              flush=True)
        if order == BIP:  # the cyclic dealing barely improves: left as it is
            tables[(W, order)] = s1
    if not args.check:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                            "svd-jacobi-mpi-cuda_amd", "csrc", "hip", "evd_deal_tables.hpp")
        with open(path, "w") as f:
            f.write(header(tables))
        print("wrote", os.path.normpath(path))


if __name__ == "__main__":
    main()
