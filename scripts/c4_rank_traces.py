"""Diagnostic: per-trial (chi2, lambda) traces of the C4 window (stable_noout, seed 0) solved on one
rank and sharded over 2 and 4 ranks (host transport over gloo, one GPU), with the reference Huber
gate (gate_mode 0) and with its rounding residue taken as 0 (gate_mode 1), next to the oracle at
several OpenMP thread counts (its own summation-order envelope).  Writes gpurun_out/c4_rank_traces.json
and prints where each trajectory first departs from the one-rank solve.

Usage (GPU box): python scripts/c4_rank_traces.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lego-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import lego_ba  # noqa: E402
import oracle_bind as ob  # noqa: E402
from test_multirank_gpu import run_sharded  # noqa: E402
from windows import window  # noqa: E402


def summary(r):
    return dict(iterations=int(r["iterations"]), trials=int(r["trials"]), chi2_final=float(r["chi2_final"]),
                trace_chi2=[float(x) for x in r["trace_chi2"]], trace_lambda=[float(x) for x in r["trace_lambda"]])


def first_departure(a, b):
    n = min(len(a["trace_chi2"]), len(b["trace_chi2"]))
    for i in range(n):
        if abs(a["trace_chi2"][i] - b["trace_chi2"][i]) > 1e-9 * abs(b["trace_chi2"][i]):
            return i, abs(a["trace_chi2"][i] - b["trace_chi2"][i]) / abs(b["trace_chi2"][i])
    return None, 0.0


def main():
    w = window("C4", seed=0, family="stable_noout")
    out = {}
    for gate in (0, 1):
        s = lego_ba.Solver(gate_mode=gate)
        out[f"gpu_1rank_g{gate}"] = summary(s.solve(w))
        s.close()
        for world in (2, 4):
            r = run_sharded("C4", 0, "stable_noout", world=world, timeout=400, gate_mode=gate)
            out[f"gpu_{world}rank_g{gate}"] = summary(r[0])
            print(f"gate {gate} world {world} done", flush=True)
        for t in (1, 2, 4, 8, 16):
            out[f"oracle_t{t}_g{gate}"] = summary(ob.solve(w, n_threads=t, gate_mode=gate))
            print(f"gate {gate} oracle t{t} done", flush=True)
    for k, v in out.items():
        base = out[f"gpu_1rank_g{k[-1]}"]
        i, d = first_departure(v, base)
        print(f"{k:20s} it {v['iterations']:2d} tr {v['trials']:2d} chi2 {v['chi2_final']:.10f} "
              f"first departure from 1-rank at trace entry {i} (rel {d:.2e})")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "c4_rank_traces.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
