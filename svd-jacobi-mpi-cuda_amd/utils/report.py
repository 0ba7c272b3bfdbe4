"""Run reports.

* :func:`reference_report_text` / :func:`write_reference_report` -- the
  reference's text report ``reporte-dimension-<n>-time-<dd-mm-YYYY-HH-MM-SS>.txt``
  with the same lines it prints (reference main.cu:1539-1545, 1581-1584,
  1637-1638, 1664-1669).  The reference's "Number of threads" line always
  read 1 (omp_get_num_threads outside a parallel region, main.cu:1581); here
  it reports the real worker count (GPUs, or CPU threads for the oracle).
* :func:`run_record` / :func:`write_json` -- structured JSON with sweeps,
  per-sweep off values, times, GFLOP/s and accuracy (SURVEY.md section 5,
  "Metrics / logging / observability").
"""
from __future__ import annotations

import datetime
import json
import os
import platform

from .metrics import algorithmic_flops_per_sweep


def timestamp() -> str:
    return datetime.datetime.now().strftime("%d-%m-%Y-%H-%M-%S")


def reference_report_text(m: int, n: int, seconds: float, residual: float | None,
                          workers: int) -> str:
    lines = [f"Number of threads: {workers}",
             f"Dimensions, height: {m}, width: {n}",
             f"SVD MPI+OMP time with U,V calculation: {seconds}"]
    if residual is not None:
        lines.append(f"||A-USVt||_F: {residual}")
    return "\n".join(lines) + "\n"


def write_reference_report(directory: str, m: int, n: int, seconds: float,
                           residual: float | None, workers: int) -> str:
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, f"reporte-dimension-{m}-time-{timestamp()}.txt")
    with open(path, "w") as f:
        f.write(reference_report_text(m, n, seconds, residual, workers))
    return path


def run_record(result, m: int, n: int, n_gpus: int, accuracy: dict | None = None,
               extra: dict | None = None) -> dict:
    sweeps = int(result.sweeps)
    secs = float(result.seconds)
    rec = {
        "m": m, "n": n, "n_gpus": n_gpus, "method": result.method,
        "sweeps": sweeps, "converged": bool(result.info.get("converged", False)),
        "seconds": secs,
        "gflops_algorithmic": result.info.get("flops", algorithmic_flops_per_sweep(m, n) * sweeps)
        / max(secs, 1e-12) / 1e9,
        "off_history": [float(h) for h in result.history],
        "info": {k: (v if isinstance(v, (int, float, str, bool, list, dict, type(None))) else str(v))
                 for k, v in result.info.items()},
        "host": platform.node(),
        "time": timestamp(),
    }
    if accuracy:
        rec["accuracy"] = accuracy
    if extra:
        rec.update(extra)
    return rec


def write_json(path: str, record: dict) -> str:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        json.dump(record, f, indent=2, default=str)
    return path
