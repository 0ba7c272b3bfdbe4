"""Spread exchange: a tournament round's point-to-point transfer over ALL xGMI
links of the node, relayed in two phases.

In a round of the tournament every GPU sends one half super-block to one peer
and receives one from another (a permutation).  Sent directly, the transfer
uses ONE of a GPU's seven xGMI links (MI355X: 7 links per GPU, fully
connected 8-GPU node) while the other six idle; at n = 16384 on 8 GPUs a
half is 67 MB, about 1 ms per link direction, and the next round's first
task waits for it (README "Multi-GPU on a one-GPU box").  The reference's
exchange is a host-staged star through rank 0 (main.cu:582-680, 854-936).

Here a message from s to d = send_to[s] is cut into P - 1 chunks:

* chunk 0 goes directly s -> d (phase 1);
* chunk j >= 1 goes to relay q_j (the j-th rank not in {s, d}) in phase 1
  and is forwarded q_j -> d in phase 2.

Because send_to is a permutation, in each phase every directed link carries
at most one chunk per message: a relay forwards for P - 2 sources whose
destinations are distinct.  With links of equal speed the exchange takes
2 / (P - 1) of the direct time (8 GPUs: 0.29x), at the cost of one extra
hop per byte and (P - 2) chunk-sized relay buffers per message.

Both phases are grouped RCCL send/recv batches on the comm stream, phase 2
stream-ordered after phase 1, so the relay's forwards read what it received.
Between any two ranks, within a phase and a direction, both sides enumerate
their ops message by message in the same order (one op per message), which
is the order RCCL matches sends and receives in.
"""
from __future__ import annotations

from dataclasses import dataclass


def relays(P: int, s: int, d: int) -> list:
    """Relay ranks of the message s -> d, in chunk order (chunk j -> relays[j-1])."""
    return [q for q in range(P) if q != s and q != d]


def chunk_bounds(n: int, parts: int) -> list:
    """[(begin, end)] of ``parts`` near-equal contiguous pieces of n elements."""
    base, rem = divmod(n, parts)
    out, a = [], 0
    for j in range(parts):
        b = a + base + (1 if j < rem else 0)
        out.append((a, b))
        a = b
    return out


@dataclass
class SpreadOps:
    """Ops of one rank for one exchange: lists of (message index, (begin,
    end) element range, peer, where) with ``where`` = "out" (the outgoing
    message), "in" (the incoming one) or ("relay", source rank)."""
    p1_send: list
    p1_recv: list
    p2_send: list
    p2_recv: list


def spread_ops(rank: int, send_to, sizes: list, spread: list) -> SpreadOps:
    """The two phases of rank ``rank`` for messages of ``sizes`` elements
    (``spread[i]`` False: message i goes directly, e.g. the tiny norms).
    ``send_to[s]`` is the destination of rank s in this round."""
    P = len(send_to)
    g = rank
    recv_from = [0] * P
    for s in range(P):
        recv_from[int(send_to[s])] = s
    dst, src = int(send_to[g]), recv_from[g]
    ops = SpreadOps([], [], [], [])
    for mi, n in enumerate(sizes):
        if not spread[mi] or P <= 2:
            ops.p1_send.append((mi, (0, n), dst, "out"))
            ops.p1_recv.append((mi, (0, n), src, "in"))
            continue
        nb = chunk_bounds(n, P - 1)
        ops.p1_send.append((mi, nb[0], dst, "out"))
        for j, q in enumerate(relays(P, g, dst), 1):
            ops.p1_send.append((mi, nb[j], q, "out"))
        ops.p1_recv.append((mi, nb[0], src, "in"))
        for s in range(P):  # sources this rank relays for (not itself, not its own sender)
            if s == g or s == src:
                continue
            d = int(send_to[s])
            j = relays(P, s, d).index(g) + 1
            ops.p1_recv.append((mi, nb[j], s, ("relay", s)))
            ops.p2_send.append((mi, nb[j], d, ("relay", s)))
        for j, q in enumerate(relays(P, src, g), 1):
            ops.p2_recv.append((mi, nb[j], q, "in"))
    return ops


def relay_chunk(n: int, P: int) -> int:
    """Largest chunk of an n-element message (relay buffer size per source)."""
    return -(-n // (P - 1)) if P > 2 else 0


def modelled_time_factor(P: int) -> float:
    """Transfer time of a spread exchange relative to a direct one, links of
    equal speed, both phases bandwidth-bound."""
    return 2.0 / (P - 1) if P > 2 else 1.0


EXCHANGES = ("auto", "direct", "spread")


def resolve_exchange(mode: str, P: int) -> str:
    """``auto``: spread from 4 GPUs up (3 GPUs gain nothing: 2 chunks, two
    phases), direct below."""
    if mode not in EXCHANGES:
        raise ValueError(f"exchange must be one of {EXCHANGES}, got {mode!r}")
    if mode == "auto":
        return "spread" if P >= 4 else "direct"
    return mode if P > 2 else "direct"
