"""Sweep-level checkpoint / resume.

The reference has none.  The whole solver state after a
sweep is small and self-contained: the resident columns of A and V, the
tracked squared norms D, the sweep index / history and (distributed) the
super-block placement.  One file per rank; written atomically; loaded with
``torch.load(weights_only=True)`` (only tensors and plain Python values are
stored).
"""
from __future__ import annotations

import os

import torch


def path_for(directory: str, rank: int) -> str:
    return os.path.join(directory, f"svdj_ckpt_rank{rank}.pt")


def save(directory: str, rank: int, state: dict) -> str:
    os.makedirs(directory, exist_ok=True)
    path = path_for(directory, rank)
    tmp = path + ".tmp"
    cpu_state = {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in state.items()}
    torch.save(cpu_state, tmp)
    os.replace(tmp, path)
    return path


def load(directory: str, rank: int, device=None) -> dict | None:
    path = path_for(directory, rank)
    if not os.path.exists(path):
        return None
    st = torch.load(path, map_location="cpu", weights_only=True)
    if device is not None:
        st = {k: (v.to(device) if torch.is_tensor(v) else v) for k, v in st.items()}
    return st


def compatible(state: dict, signature: dict) -> bool:
    """A checkpoint is resumable only for the same problem/geometry."""
    return all(state.get(k) == v for k, v in signature.items())


def clear(directory: str, rank: int):
    p = path_for(directory, rank)
    if os.path.exists(p):
        os.remove(p)
