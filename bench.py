"""bench.py — LM iterations/s and ms/solve of the MI355X BA solver.

A "step" is one complete Backend::Optimize solve (problem.solve(10),
src/backend_lego.cpp:161) of a device-resident sliding window: restart from the
uploaded initial state, run every LM trial to the reference stop rule.
value = LM iterations completed per second, summed over ranks.

Workload (BASELINE.json metric window, configs[2]): 20 keyframes, 50 000
landmarks, 400 000 observations per GPU, fp64 throughout (>= the reference's
double).  With N GPUs the window grows to N x 50 000 landmarks (landmark
shards, poses replicated, one RCCL all-reduce of the reduced pose system per
LM trial) -> "scaling": "weak"; value counts shard-iterations (iterations x N).

Usage: python bench.py [--gpus N --steps K --warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lego-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import lego_ba  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec
FP64_PEAK_TFS = 78.6       # MI355X FP64 spec (vector = matrix); measured on the box:
                           # v_mfma_f64_16x16x4 72.0 TF, v_fma_f64 60.5 TF (lego-slam_amd/tools/ubench_fp64_peak.hip)
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r01_pmc_k_lin.json")


def survey_bytes_per_iteration(n_obs, n_lm):
    """SURVEY.md 8(d) compulsory HBM bytes of one LM iteration (one k_lin launch fuses the
    three passes: linearise + Schur, back-substitute, chi2-evaluate):
    B = 3 (12 O + 28 L) + 24 L."""
    return 3 * (12 * n_obs + 28 * n_lm) + 24 * n_lm


def survey_flops_per_iteration(n_obs, n_lm, k):
    """SURVEY.md 8(d) fp64 flops of one LM iteration: 400 O (projection, Jacobians, J^T W J,
    H_pl H_ll^-1) + 216 sum_l k(k+1)/2 (Schur pair blocks) + 50 L (3x3 inverse) + 80 O
    (back-substitution + chi2); the 6P x 6P solve (k_ctrl) is excluded."""
    return 400 * n_obs + 216 * n_lm * k * (k + 1) / 2 + 50 * n_lm + 80 * n_obs


def pmc_traffic(cfg_key):
    """HBM bytes per k_lin launch from the committed rocprofv3 PMC passes (scripts/gpu_pmc.sh ->
    scripts/pmc_traffic.py): 2 x FETCH_SIZE (gfx950 reports half of wide reads) + WRITE_SIZE,
    or None when no pass for this workload is committed."""
    try:
        with open(PMC_TRAFFIC) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return d.get("bytes_per_launch") if d.get("workload") == cfg_key else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--landmarks", type=int, default=50000, help="landmarks per GPU")
    ap.add_argument("--poses", type=int, default=20)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--family", default="stable_noout", choices=["stable_noout", "stable", "default"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="length of the cpu_baseline sample")
    ap.add_argument("--trials-per-sync", type=int, default=0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world != 1:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}")

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)

    from windows import STABLE
    params = dict(STABLE) if args.family.startswith("stable") else {}
    if args.family == "stable_noout":
        params["outlier_frac"] = 0.0
    L = args.landmarks
    w = lego_ba.generate_window(P=args.poses, L=L * world, k=args.k, seed=args.seed,
                                lm_begin=rank * L, lm_end=(rank + 1) * L, **params)
    if args.family.startswith("stable"):
        f = np.zeros(args.poses, np.uint8)
        f[0] = 1
        w["pose_fixed"] = f

    comm_id = bytes(128)
    if world > 1:
        obj = [lego_ba.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    solver = lego_ba.Solver(device=local, world_size=world, rank=rank, comm_id=comm_id,
                            trials_per_sync=args.trials_per_sync)
    solver.upload(w)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        solver.solve_resident()

    def timed(profile):
        solver.set_profiling(profile)
        solver.kernel_stats_reset()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        it = tr = 0
        res = None
        for _ in range(args.steps):
            res = solver.solve_resident()
            it += res["iterations"]
            tr += res["trials"]
        torch.cuda.synchronize()
        barrier()
        dt = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt, it, tr, res

    # ---- timed region: K whole solves, no per-kernel instrumentation ----
    dt, iters, trials, last = timed(False)
    # ---- the same K solves again with a HIP event pair around every kernel (on the solver's
    #      stream): per-kernel average durations for the roofline ----
    dt_prof, _, _, _ = timed(True)
    ks = solver.kernel_stats()
    solver.set_profiling(False)
    event_floor_ms = solver.event_floor_ms()   # the same event bracket around an empty kernel

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    value = world * iters / dt
    n_obs, n_lm = len(w["obs_pose"]), len(w["lm_xyz"])
    lin_n, lin_ms = ks.get("k_lin", (0, 0.0))
    lin_bracket_ms = lin_ms / max(lin_n, 1)
    # the event pair brackets the launch too: its empty-kernel floor is subtracted (rocprofv3's
    # kernel-trace average of the same command is committed under profiles/ for comparison)
    lin_avg_ms = max(lin_bracket_ms - event_floor_ms, 1e-6)
    flops_per = survey_flops_per_iteration(n_obs, n_lm, args.k)
    bytes_per = survey_bytes_per_iteration(n_obs, n_lm)
    achieved_tfs = flops_per / (lin_avg_ms * 1e-3) / 1e12 if lin_avg_ms > 0 else 0.0
    achieved_gbs = bytes_per / (lin_avg_ms * 1e-3) / 1e9 if lin_avg_ms > 0 else 0.0
    cfg_key = f"P{args.poses}-L{L}-k{args.k}-{args.family}-s{args.seed}"
    traffic = pmc_traffic(cfg_key)

    out = {
        "metric": "LM iterations/sec + ms/solve, 20KF/50k-pts/400k-obs window; final chi2 vs ref",
        "value": round(value, 3),
        "unit": "LM iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "ms_per_step_with_kernel_events": round(dt_prof / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic (tools/window_gen.c, family={args.family}, seed={args.seed})",
        "config": {"workload": f"sliding-window BA solve(10): {args.poses} KF / {L * world} landmarks / "
                               f"{n_obs * world} obs ({L} landmarks per GPU)",
                   "keyframes": args.poses, "landmarks_per_gpu": L, "obs_per_gpu": n_obs,
                   "parallelism": f"landmark-shard x{world}"},
        "iterations_per_solve": iters / args.steps,
        "trials_per_solve": trials / args.steps,
        "chi2_final": last["chi2_final"],
        "kernels_ms_per_solve": {k: round(v[1] / args.steps, 4) for k, v in ks.items()},
        # dominant kernel k_lin (one launch = one LM iteration's linearise/back-substitute/chi2 pass);
        # the path is FP64-bound (~29 flop/B > ridge 9.8 flop/B)
        "roofline": {"bound": "mfma", "achieved": round(achieved_tfs, 3), "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": round(achieved_tfs / FP64_PEAK_TFS, 4), "traffic": traffic,
                     "kernel": "k_lin", "avg_launch_ms": round(lin_avg_ms, 5), "event_bracket_ms": round(lin_bracket_ms, 5),
                     "event_floor_ms": round(event_floor_ms, 5), "flops_per_launch": flops_per,
                     "peak_note": "FP64 spec (vector = matrix); measured here 72.0 TF MFMA, 60.5 TF VALU"},
        "roofline_hbm": {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": bytes_per,
                         "traffic": traffic},
    }
    # the same window through the PCG reduced solve (BASELINE config 3 names "Schur + PCG"; the
    # reference's own solver, and value above, is the LDLT): reported beside value, never as it
    if world == 1:
        sp = lego_ba.Solver(device=local, linear_solver=lego_ba.LH_SOLVER_PCG)
        sp.upload(w)
        sp.solve_resident()
        torch.cuda.synchronize()
        t = time.perf_counter()
        pits = pcgs = 0
        for _ in range(args.steps):
            r = sp.solve_resident()
            pits += r["iterations"]
            pcgs += r["pcg_iterations"]
        torch.cuda.synchronize()
        dtp = time.perf_counter() - t
        out["pcg"] = {"ms_per_solve": round(dtp / args.steps * 1e3, 4), "iterations_per_s": round(pits / dtp, 3),
                      "iterations_per_solve": pits / args.steps, "pcg_steps_per_solve": pcgs / args.steps,
                      "chi2_rel_vs_ldlt": abs(r["chi2_final"] - last["chi2_final"]) / last["chi2_final"]}
        sp.close()
    # the frontend's pose-only LM (Frontend::EstimateCurrentPose) on a batch of
    # frames through lh_estimate_pose: device time of one launch over the batch, beside value
    if world == 1:
        import frames
        nf = 2048
        fb = frames.batch(args.seed, nf, n_obs=150)
        sf = lego_ba.Solver(device=local)
        sf.estimate_pose(fb)
        tms = [sf.estimate_pose(fb)["time_ms"] for _ in range(3)]
        out["estimate_pose"] = {"frames": nf, "obs_per_frame": 150, "ms_per_batch": round(min(tms), 4),
                                "frames_per_s": round(nf / (min(tms) * 1e-3), 1),
                                "note": "device time of one lh_estimate_pose launch (4 rounds of solve(10) per frame)"}
        if not args.no_cpu:
            import oracle_bind
            t = time.perf_counter()
            oracle_bind.estimate_pose(frames.batch(args.seed, 256, n_obs=150))
            out["estimate_pose"]["cpu_frames_per_s_1core"] = round(256 / (time.perf_counter() - t), 1)
        sf.close()
    # end-to-end host-buffer call (lh_solve: upload + solve + download over PCIe), rank 0 only
    if world == 1:
        solver_h = lego_ba.Solver(device=local)
        solver_h.solve(w)
        t = time.perf_counter()
        solver_h.solve(w)
        out["ms_per_solve_host_buffers"] = round((time.perf_counter() - t) * 1e3, 3)
        solver_h.close()
    if world == 1 and not args.no_cpu:
        import oracle_bind
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        # bounded sample: repeated full solves of the same window for >= cpu_seconds of CPU work
        t = time.perf_counter()
        its = nsolve = 0
        while True:
            o = oracle_bind.solve(w, n_threads=threads)
            its += o["iterations"]
            nsolve += 1
            ct = time.perf_counter() - t
            if ct >= args.cpu_seconds:
                break
        out["cpu_baseline"] = {"value": round(its / ct, 4), "unit": "LM iterations/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{nsolve} full solve(10)s of the same window by the block-sparse oracle "
                                         f"(oracle/lego_oracle.c ref_sparse, OpenMP {threads} threads), {ct:.1f} s, "
                                         f"{its} iterations"}
        out["chi2_rel_vs_oracle"] = abs(last["chi2_final"] - o["chi2_final"]) / o["chi2_final"]
        out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 2)
    print(json.dumps(out))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
