"""bench.py — LM iterations/s and ms/solve of the MI355X BA solver.

A "step" is one complete Backend::Optimize solve (problem.solve(10), src/backend_lego.cpp:161) of a
device-resident sliding window: restart from the uploaded initial state, run every LM trial to the
reference stop rule.  value = LM iterations (of the whole window) completed per second.

Workloads (BASELINE.json configs); fp64 throughout (>= the reference's double):
  C3  20 KF / 50 000 landmarks / 400 000 obs on one GPU: the metric window (the N = 1 default).
  C4  BASELINE config 4, the N > 1 default: 20 KF / 500 000 landmarks / 4 000 000 obs, landmark-sharded
      over the N GPUs (poses replicated, one RCCL all-reduce of the reduced pose system per LM trial),
      the same window at every N ("scaling": "strong").  value counts C3-equivalent work: C4 has exactly 10x
      C3's landmarks and observations, so value = 10 x (LM iterations of C4) / s over the max-over-ranks time,
      in the unit of the N = 1 line.  The driver's value(N) / value(1) therefore compares C4 on N GPUs with C3
      on one, which flatters the ratio (one GPU solves C4 at ~1.9x C3's C3-equivalent rate: the controller's
      fixed cost per trial is amortised over 10x the landmarks); the strong-scaling figure is
      c4_speedup_vs_1gpu beside value: C4's iterations/s on N GPUs over C4's on one GPU of the same job (rank 0
      alone, measured after the timed region).  C4 runs in gate_mode 1 (the Huber gate's analytically-zero
      rounding residue taken as 0): with the reference gate its trajectory depends on the summation order, hence
      on the rank count (the oracle alone ends after 4 or 7 iterations depending on its thread count,
      profiles/r03_c4_oracle_gate_envelope.json); in gate_mode 1 every rank count runs the same trajectory
      (tests/test_multirank_gpu.py).  The N = 1 line carries C4 on one GPU ("c4_1gpu") and each rank's share of
      C4 sharded 2, 4 and 8 ways solved alone ("c4_shards_1gpu": the per-rank work without the all-reduce).
  C3w (--workload C3w, a side measurement, never the default) one C3-sized shard per GPU: a window of
      50 000 N landmarks ("scaling": "weak"), value = N x (LM iterations of the window) / s.

Usage: python bench.py [--gpus N --steps K --warmup W] [--workload C3|C3w|C4]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lego-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import lego_ba  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec
FP64_PEAK_TFS = 78.6       # MI355X FP64 spec (vector = matrix); measured on the box:
                           # v_mfma_f64_16x16x4 72.0 TF, v_fma_f64 60.5 TF (lego-slam_amd/tools/ubench_fp64_peak.hip)
# the committed rocprofv3 evidence of this tree's k_lin (LH_PMC_JSON / LH_ROCPROF_JSON: the same files written
# earlier in the same GPU call, before they are committed)
PMC_TRAFFIC = os.environ.get("LH_PMC_JSON", os.path.join(ROOT, "profiles", "r06ak_pmc_k_lin.json"))
ROCPROF_K_LIN = os.environ.get("LH_ROCPROF_JSON", os.path.join(ROOT, "profiles", "r06av_rocprof_k_lin.json"))
# L: landmarks of the window; per_rank: L per rank (the window has L N landmarks; weak scaling)
WORKLOADS = {"C3": dict(P=20, L=50_000, k=8), "C3w": dict(P=20, L=50_000, k=8, per_rank=True),
             "C4": dict(P=20, L=500_000, k=8)}


def default_workload(world):
    """The contract line's workload: C3 (the metric window) on one GPU, BASELINE config 4's C4 past it."""
    return "C3" if world == 1 else "C4"


def c3_units(name, world):
    """value's unit is one LM iteration of a C3-sized window: a window of L landmarks (k observations each,
    the same keyframes) counts L / 50 000 of them (C4: 10; C3w: N)."""
    c = WORKLOADS[name]
    L = c["L"] * world if c.get("per_rank") else c["L"]
    return L / WORKLOADS["C3"]["L"]


def survey_bytes_per_iteration(n_obs, n_lm):
    """SURVEY.md 8(d) compulsory HBM bytes of one LM iteration (one k_lin launch fuses the three
    passes: linearise + Schur, back-substitute, chi2-evaluate): B = 3 (12 O + 28 L) + 24 L."""
    return 3 * (12 * n_obs + 28 * n_lm) + 24 * n_lm


def survey_flops_per_iteration(n_obs, n_lm, k):
    """SURVEY.md 8(d) fp64 flops of one LM iteration: 400 O (projection, Jacobians, J^T W J,
    H_pl H_ll^-1) + 216 sum_l k(k+1)/2 (Schur pair blocks) + 50 L (3x3 inverse) + 80 O
    (back-substitution + chi2); the 6P x 6P solve (k_ctrl) is excluded."""
    return 400 * n_obs + 216 * n_lm * k * (k + 1) / 2 + 50 * n_lm + 80 * n_obs


def pmc_traffic(cfg_key):
    """HBM bytes per k_lin launch from the committed rocprofv3 PMC passes (scripts/gpu.sh pmc ->
    scripts/pmc_traffic.py): 2 x FETCH_SIZE (gfx950 reports half of wide reads) + WRITE_SIZE,
    or None when no pass for this workload is committed."""
    try:
        with open(PMC_TRAFFIC) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return d.get("bytes_per_launch") if d.get("workload") == cfg_key else None


def cgroup_cpus():
    """CPUs this process may actually use per the cgroup CPU quota (cpu.max: "quota period"), or
    None without a quota.  A GPU box exposes every core of the host in its affinity mask (256)
    but grants the job a share of them through the quota."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                return max(1, -(-int(q) // int(per)))
        except (OSError, ValueError):
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def host_info():
    """The host the CPU baseline ran on: core counts and CPU model, and the
    thread count the baseline uses: every CPU this process may use (affinity mask capped by the
    cgroup quota; without a quota, by OMP_NUM_THREADS when the job sets one)."""
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = cgroup_cpus()
    omp = os.environ.get("OMP_NUM_THREADS")
    usable = avail
    if quota is not None:
        usable = min(usable, quota)
    elif omp and omp.isdigit() and int(omp) > 0:
        usable = min(usable, int(omp))
    return {"nproc": os.cpu_count(), "cpus_in_affinity_mask": avail, "cgroup_cpu_quota": quota,
            "omp_num_threads_env": omp, "cpus_usable": usable, "cpu_model": model}


def native_oracle():
    """The timed CPU baseline build: the oracle at -O3 -march=native, compiled
    here for this host's CPU (the parity build in oracle/ is portable).  -ffp-contract=off keeps the
    reference's roundings (no FMA), so it computes the same numbers.  Falls back to the parity build."""
    src = [os.path.join(ROOT, "oracle", "lego_oracle.c"), os.path.join(ROOT, "oracle", "lk_oracle.c")]
    out = os.path.join(tempfile.gettempdir(), f"liblego_oracle_native_{os.getpid()}.so")
    flags = ["-O3", "-march=native", "-fPIC", "-std=gnu11", "-ffp-contract=off", "-fopenmp", "-shared"]
    try:
        subprocess.run(["gcc", *flags, "-o", out, *src, "-lm"], check=True, timeout=120, capture_output=True)
        return out, " ".join(flags)
    except (OSError, subprocess.SubprocessError):
        return None, "-O3 -ffp-contract=off -fopenmp (parity build; native build failed)"


def cxx_caller_ms(w, reps, exe=None, line=False, env=None, both=False):
    """Median wall time of lh_solve on this window from the compiled C++ caller (tests/abi_caller.cpp,
    window file format there), or None when the binary is missing or fails.  line: return the caller's
    whole timing line (prep / upload / solve / download of the last call) instead.  both: a pair, the
    call that downloads the per-edge chi2 and the call with the outlier pass on the device (flags only;
    None unless its flags equal the host pass's)."""
    exe = exe or os.path.join(ROOT, "lego-slam_amd", "lib", "abi_caller")
    if not os.path.exists(exe):
        return None if not both else (None, None)
    O = len(w["obs_pose"])
    ext = w.get("cam_ext")
    fixed = w.get("pose_fixed")
    with tempfile.TemporaryDirectory() as td:
        win, res = os.path.join(td, "w.bin"), os.path.join(td, "r.bin")
        with open(win, "wb") as f:
            np.array([len(w["pose_Tcw"]), len(w["lm_xyz"])], np.int32).tofile(f)
            np.array([O], np.int64).tofile(f)
            np.array([0 if ext is None else len(ext), 0 if fixed is None else 1], np.int32).tofile(f)
            np.asarray(w["K"], np.float64).tofile(f)
            np.asarray(w["pose_Tcw"], np.float64).tofile(f)
            if fixed is not None:
                np.asarray(fixed, np.uint8).tofile(f)
            np.asarray(w["lm_xyz"], np.float64).tofile(f)
            np.asarray(w["obs_pose"], np.uint32).tofile(f)
            np.asarray(w["obs_lm"], np.uint32).tofile(f)
            np.asarray(w["obs_cam"] if w.get("obs_cam") is not None else np.zeros(O), np.uint8).tofile(f)
            np.asarray(w["obs_uv"], np.float64).tofile(f)
            if ext is not None:
                np.asarray(ext, np.float64).tofile(f)
        try:
            r = subprocess.run([exe, win, res, str(reps)], capture_output=True, text=True, timeout=120,
                               env=None if env is None else {**os.environ, **env})
        except subprocess.TimeoutExpired:
            return None
        out = {}
        for ln in r.stdout.splitlines():
            if "lh_solve median" in ln:
                key = "device" if "device outlier pass" in ln else "chi2"
                ok = key == "chi2" or "flags equal" in ln
                out[key] = ln if line else (round(float(ln.split("lh_solve median")[1].split()[0]), 3) if ok else None)
        return out.get("chi2") if not both else (out.get("chi2"), out.get("device"))
    return None if not both else (None, None)


def make_window(name, family, seed, rank, world):
    """Rank `rank`'s landmark shard of workload `name` (all of it with world = 1), generated directly."""
    from windows import STABLE
    c = WORKLOADS[name]
    params = {}
    if family.startswith("stable"):
        params.update(STABLE)
    if family == "stable_noout":
        params["outlier_frac"] = 0.0
    L = c["L"] * world if c.get("per_rank") else c["L"]
    w = lego_ba.generate_window(P=c["P"], L=L, k=c["k"], seed=seed, lm_begin=rank * L // world,
                                lm_end=(rank + 1) * L // world, **params)
    if family.startswith("stable"):
        f = np.zeros(c["P"], np.uint8)
        f[0] = 1
        w["pose_fixed"] = f
    return w


def time_solves(solver, steps, barrier):
    import torch
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    it = tr = 0
    res = None
    for _ in range(steps):
        res = solver.solve_resident()
        it += res["iterations"]
        tr += res["trials"]
    torch.cuda.synchronize()
    barrier()
    return time.perf_counter() - t0, it, tr, res


def rocprof_k_lin(cfg_key):
    """k_lin durations from the committed rocprofv3 kernel trace of this bench (scripts/rocprof_k_lin.py):
    the same back-to-back replays the live timing uses, and the launches inside the timed solves."""
    try:
        with open(ROCPROF_K_LIN) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return d if d.get("workload") == cfg_key else None


def roofline(solver, n_obs, n_lm, k, cfg_key, reps=50):
    """k_lin (the dominant kernel; one launch = one LM trial's linearise / back-substitute / chi2 pass)
    against the FP64 peak: SURVEY 8(d) flops per iteration / k_lin's duration, the latter measured by
    replaying the solve's trial-mode launch `reps` times back to back between HIP events on the
    solver's stream (lh_debug_time_lin)."""
    ms = solver.time_lin_ms(reps)
    flops = survey_flops_per_iteration(n_obs, n_lm, k)
    nbytes = survey_bytes_per_iteration(n_obs, n_lm)
    tfs = flops / (ms * 1e-3) / 1e12
    gbs = nbytes / (ms * 1e-3) / 1e9
    traffic = pmc_traffic(cfg_key)
    rl = {"bound": "mfma", "achieved": round(tfs, 3), "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
          "frac": round(tfs / FP64_PEAK_TFS, 4), "traffic": traffic, "kernel": "k_lin",
          "avg_launch_ms": round(ms, 5), "timing": f"{reps} back-to-back replays between HIP events on the solver's stream",
          "flops_per_launch": flops,
          "peak_note": "FP64 spec (vector = matrix); measured here 72.0 TF MFMA, 60.5 TF VALU"}
    rp = rocprof_k_lin(cfg_key)
    if rp:
        # the committed kernel trace of the same command: its replay launches (must agree with
        # avg_launch_ms) and the k_lin launches inside the solves (after k_ctrl, a few us slower)
        rl["rocprof_replay_avg_ms"] = round(rp["replay_avg_us"] * 1e-3, 5)
        rl["rocprof_in_solve_avg_ms"] = round(rp["in_solve_avg_us"] * 1e-3, 5)
        rl["frac_in_solve_rocprof"] = round(flops / (rp["in_solve_avg_us"] * 1e-6) / 1e12 / FP64_PEAK_TFS, 4)
    return (rl,
            {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": nbytes, "traffic": traffic})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 1000 C3 solves is ~1.1 s of GPU work: long enough for the driver's utilisation sampling to see it
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="auto", choices=["auto", "C3", "C3w", "C4"],
                    help="auto: C3 on one GPU, C4 (BASELINE config 4, landmark-sharded, strong scaling) over N > 1")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--family", default="stable_noout", choices=["stable_noout", "stable", "default"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-extras", action="store_true", help="only the timed line (no side measurements)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="length of the cpu_baseline sample")
    ap.add_argument("--trials-per-sync", type=int, default=0)
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host", "p2p"],
                    help="per-trial exchange with N > 1: RCCL over xGMI (the default), the one-shot peer-write "
                         "exchange on the device (LH_COMM_P2P: IPC-mapped buffers, bootstrap over gloo), or the "
                         "ABI's host transport over gloo (a rehearsal of the N-rank flow on fewer GPUs)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world != 1:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}")
    name = args.workload if args.workload != "auto" else default_workload(world)

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    ndev = max(1, torch.cuda.device_count())
    if world > 1 and args.comm == "rccl" and ndev < world:
        raise SystemExit(f"{world} ranks need {world} GPUs for RCCL (found {ndev}); --comm host or p2p rehearse on fewer")
    local = local % ndev
    torch.cuda.set_device(local)

    w = make_window(name, args.family, args.seed, rank, world)
    gate = 1 if name == "C4" else 0
    comm_id = bytes(128)
    extra = {}
    if world > 1 and args.comm == "rccl":
        obj = [lego_ba.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    elif world > 1:
        def allreduce(buf, op):
            t = torch.from_numpy(buf)   # the library's pinned exchange buffer
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX)
        extra = dict(allreduce=allreduce)
        if args.comm == "p2p":
            extra["comm_mode"] = lego_ba.LH_COMM_P2P
    solver = lego_ba.Solver(device=local, world_size=world, rank=rank, comm_id=comm_id, gate_mode=gate,
                            trials_per_sync=args.trials_per_sync, **extra)
    solver.upload(w)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        solver.solve_resident()
    # ---- timed region: K whole solves of the resident window, no per-kernel instrumentation ----
    dt, iters, trials, last = time_solves(solver, args.steps, barrier)
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # the same solves with a HIP event pair around every kernel: per-kernel ms per solve
    solver.set_profiling(True)
    solver.kernel_stats_reset()
    time_solves(solver, max(2, min(20, args.steps // 4)), barrier)
    ks = solver.kernel_stats()
    solver.set_profiling(False)
    n_obs, n_lm = len(w["obs_pose"]), len(w["lm_xyz"])
    c = WORKLOADS[name]
    cfg_key = f"{name}-{args.family}-s{args.seed}" + (f"-x{world}" if WORKLOADS[name].get("per_rank") else "")
    rl, rl_hbm = roofline(solver, n_obs, n_lm, c["k"], cfg_key)

    # C4 on N > 1 GPUs: the same window on rank 0's GPU alone (one rank, the same gate mode and trajectory), the
    # base of c4_speedup_vs_1gpu; the other ranks wait at the barrier below
    c4_one = None
    if name == "C4" and world > 1 and rank == 0:
        w1 = make_window("C4", args.family, args.seed, 0, 1)
        s1 = lego_ba.Solver(device=local, gate_mode=1, trials_per_sync=args.trials_per_sync)
        s1.upload(w1)
        for _ in range(2):
            s1.solve_resident()
        n1 = max(5, min(20, args.steps // 10))
        d1, i1, t1, l1 = time_solves(s1, n1, lambda: None)
        c4_one = {"iterations_per_s": round(i1 / d1, 3), "ms_per_solve": round(d1 / n1 * 1e3, 3),
                  "iterations_per_solve": i1 / n1, "trials_per_solve": t1 / n1, "solves": n1,
                  "chi2_final": l1["chi2_final"]}
        s1.close()
        del w1

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    weak = bool(WORKLOADS[name].get("per_rank"))
    L_win = c["L"] * world if weak else c["L"]
    # the unit: one LM iteration of a C3-sized window (C4 counts 10 per iteration, C3w N)
    units = c3_units(name, world)
    value = iters * units / dt
    nprof = max(2, min(20, args.steps // 4))
    out = {
        "metric": "LM iterations/sec + ms/solve, 20KF/50k-pts/400k-obs window; final chi2 vs ref",
        "value": round(value, 3),
        "unit": "LM iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        # the default series (C3 at N = 1, C4 past it): the window is fixed past N = 1; C3w fixes the per-GPU work
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic (tools/window_gen.c, family={args.family}, seed={args.seed})",
        "config": {"workload": f"{name}: sliding-window BA solve(10), {c['P']} KF / {L_win} landmarks / "
                               f"{L_win * c['k']} obs" + (f", landmark-sharded over {world} GPUs" if world > 1 else "")
                               + (" (one C3-sized shard per GPU)" if weak else ""),
                   "keyframes": c["P"], "landmarks": L_win, "landmarks_per_gpu": L_win // world,
                   "obs_this_rank": n_obs, "parallelism": f"landmark-shard x{world}",
                   "exchange": ("none" if world == 1 else {"rccl": "RCCL all-reduce",
                                                           "p2p": "one-shot peer-write exchange (LH_COMM_P2P)",
                                                           "host": "host transport over gloo (rehearsal)"}[args.comm])},
        "gate_mode": gate,
        "value_definition": ("LM iterations of the whole window per second" if units == 1.0 else
                             f"C3-equivalent LM iterations per second: {units:g} x the LM iterations of the whole "
                             f"window ({L_win} landmarks = {units:g} x C3's 50 000, the same keyframes and "
                             f"observations per landmark) over the max-over-ranks time, the unit of the N = 1 (C3) "
                             f"line" + (" (weak scaling: one C3-sized shard per GPU)" if weak else
                                        "; strong scaling: see c4_speedup_vs_1gpu")),
        "c3_units_per_iteration": units,
        "window_iterations_per_s": round(iters / dt, 3),
        "iterations_per_solve": iters / args.steps,
        "trials_per_solve": trials / args.steps,
        "trials_per_s": round(trials / dt, 3),
        "ms_per_trial": round(dt / trials * 1e3, 5),
        "chi2_final": last["chi2_final"],
        "kernels_ms_per_solve_event_bracketed": {k: round(v[1] / nprof, 4) for k, v in ks.items()},
        "roofline": rl,
        "roofline_hbm": rl_hbm,
    }
    if c4_one is not None:
        out["c4_1gpu_same_job"] = c4_one
        out["c4_speedup_vs_1gpu"] = round((iters / dt) / c4_one["iterations_per_s"], 3)
        out["c4_speedup_note"] = ("C4's LM iterations/s on the N GPUs over the same window's on rank 0's GPU alone "
                                  "(measured in this job after the timed region): the strong-scaling speedup")
    if world > 1 or args.no_extras:
        print(json.dumps(out))
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    # ---------------- side measurements (one GPU), reported beside value, never as it ----------------
    # the drop-in call Backend::Optimize pays: lh_solve on host buffers (preprocess + copies + solve +
    # download), median of 5
    sh = lego_ba.Solver(device=local)
    prev = sh.solve(w)
    runs = []
    for _ in range(5):
        t0 = time.perf_counter()
        r = sh.solve(w, reuse=prev)   # into the same output arrays, as a caller's persistent buffers
        runs.append(((time.perf_counter() - t0) * 1e3, r))
    runs.sort(key=lambda x: x[0])
    ms_h, rh = runs[2]
    cxx, cxx_dev = cxx_caller_ms(w, 15, both=True)
    # the outlier pass on the device (ABI 5): the flags come back instead of the per-edge chi2
    runs_d = []
    prev_d = sh.solve(w, outlier_chi2_th=5.991, want_edges=False)
    for _ in range(5):
        t0 = time.perf_counter()
        rd = sh.solve(w, outlier_chi2_th=5.991, want_edges=False, reuse=prev_d)
        runs_d.append(((time.perf_counter() - t0) * 1e3, rd))
    runs_d.sort(key=lambda x: x[0])
    ms_d, rd = runs_d[2]
    out["host_buffer_path"] = {"ms_per_solve": round(ms_h, 3), "iterations_per_s": round(rh["iterations"] / ms_h * 1e3, 3),
                               "cxx_caller_ms_per_solve": cxx,
                               "cxx_caller_iterations_per_s": round(rh["iterations"] / cxx * 1e3, 3) if cxx else None,
                               "device_outlier_pass": {"ms_per_solve": round(ms_d, 3), "cxx_caller_ms_per_solve": cxx_dev,
                                                       "download_ms": round(rd["time_download_ms"], 3),
                                                       "note": "the same call with Backend::Optimize's outlier pass on "
                                                               "the device (lh_result.is_outlier): flags instead of the "
                                                               "per-edge chi2 cross the link; the C++ caller checks its "
                                                               "flags against the host pass"},
                               "prep_ms": round(rh["time_prep_ms"], 3),
                               "copies_ms": round(rh["time_upload_ms"] - rh["time_prep_ms"], 3),
                               "solve_ms": round(rh["time_ms"], 3), "download_ms": round(rh["time_download_ms"], 3),
                               "note": "lh_solve(window in host memory): planner (prep) + pinned host-to-device copies + "
                                       "solve + outputs (poses, landmarks, per-edge rho) back into the caller's output arrays "
                                       "(allocated once); median of 5, from Python; cxx_caller_*: the same call from the "
                                       "compiled C++ caller (tests/abi_caller.cpp, the INTEGRATION.md flow), median of 15"}
    sh.close()
    # C4 on one GPU: the base of the N-GPU scaling ratio (SCALE lines run C4 sharded)
    if name == "C3":
        w4 = make_window("C4", args.family, args.seed, 0, 1)
        s4 = lego_ba.Solver(device=local, gate_mode=1)
        s4.upload(w4)
        for _ in range(2):
            s4.solve_resident()
        n4 = 10   # (5 solves let one host hiccup move the figure by a third)
        d4, i4, t4, l4 = time_solves(s4, n4, barrier)
        r4, _ = roofline(s4, len(w4["obs_pose"]), len(w4["lm_xyz"]), 8, f"C4-{args.family}-s{args.seed}", reps=10)
        out["c4_1gpu"] = {"gate_mode": 1, "iterations_per_s": round(i4 / d4, 3), "ms_per_solve": round(d4 / n4 * 1e3, 3),
                          "trials_per_s": round(t4 / d4, 3), "ms_per_trial": round(d4 / t4 * 1e3, 5),
                          "iterations_per_solve": i4 / n4, "trials_per_solve": t4 / n4, "chi2_final": l4["chi2_final"],
                          "k_lin_ms": r4["avg_launch_ms"], "k_lin_frac_fp64": r4["frac"]}
        s4.close()
        # the per-rank work of C4 sharded N ways, measured on this one GPU: rank 0's shard (L / N
        # landmarks, poses replicated) solved as a window of its own.  A sharded trial is k_lin + k_reduce on
        # the shard, the all-reduce of the packed reduced system (the one term a single GPU cannot measure),
        # and the same k_ctrl on every rank; the projection leaves the all-reduce out.  Numerator and
        # denominator are the same trial kind: C4 and every shard run with every trial a full one (LH_NO_EVO,
        # LH_NO_EVAL_FIRST: each trial linearises; LH_NO_LADDER: each controller factors), so ms per trial
        # is one full k_lin -> k_reduce -> k_ctrl chain (with the initial linearisation spread over the trials).
        full_env = ("LH_NO_EVO", "LH_NO_EVAL_FIRST", "LH_NO_LADDER")

        def ms_per_full_trial(win, n):
            for k in full_env:
                os.environ[k] = "1"
            so = lego_ba.Solver(device=local, gate_mode=1)
            so.upload(win)   # (the switches are read here)
            for k in full_env:
                os.environ.pop(k)
            so.solve_resident()
            dd_, ii_, tt_, _ = time_solves(so, n, barrier)
            return so, dd_ / tt_ * 1e3, tt_ / n
        s4o, base_ms, base_tr = ms_per_full_trial(w4, 5)
        s4o.close()
        shards = {"c4_1gpu_full_trials": {"ms_per_trial": round(base_ms, 5), "trials_per_solve": base_tr}}
        for n in (2, 4, 8):
            ws = make_window("C4", args.family, args.seed, 0, n)
            ss, sms, str_ = ms_per_full_trial(ws, 5)
            ss.set_profiling(True)
            ss.kernel_stats_reset()
            time_solves(ss, 3, barrier)
            kst = ss.kernel_stats()
            ss.set_profiling(False)
            rs, _ = roofline(ss, len(ws["obs_pose"]), len(ws["lm_xyz"]), 8, "", reps=20)
            per = {k: round(v[1] / max(1, v[0]), 5) for k, v in kst.items() if k in ("k_lin", "k_reduce", "k_ctrl")}
            shards[f"n{n}"] = {"landmarks": len(ws["lm_xyz"]), "obs": len(ws["obs_pose"]),
                               "ms_per_trial": round(sms, 5), "trials_per_solve": str_,
                               "ms_per_launch_event_bracketed": per,
                               "k_lin_replay_ms": rs["avg_launch_ms"], "k_lin_frac_fp64": rs["frac"],
                               "projected_speedup_excl_allreduce": round(base_ms / sms, 3)}
            ss.close()
            del ws
        out["c4_shards_1gpu"] = dict(shards, note="rank 0's share of C4 sharded N ways solved alone on this GPU "
                                     "(gate_mode 1), and C4 itself, every trial a full one (LH_NO_EVO, "
                                     "LH_NO_EVAL_FIRST, LH_NO_LADDER); projected speedup = C4's ms per full trial / "
                                     "the shard's, the per-trial all-reduce excluded (unmeasurable on one GPU)")
        del w4
    # survey-default family (the reference's live configuration: free gauge, 2 % outliers, left image
    # only).  Its C3 windows have landmarks running off to ~1e15 and are not reproducible under
    # summation reorders even in the oracle; seed 5 is, with the Huber-gate residue
    # taken as 0 on both sides (gate_mode 1): parity is checked on it.
    wd = make_window("C3", "default", 5, 0, 1)
    sd = lego_ba.Solver(device=local, gate_mode=1)
    sd.upload(wd)
    sd.solve_resident()
    dd, idd, tdd, ld = time_solves(sd, 5, barrier)
    out["survey_default_c3"] = {"seed": 5, "gate_mode": 1, "iterations_per_s": round(idd / dd, 3),
                                "ms_per_solve": round(dd / 5 * 1e3, 3), "iterations_per_solve": idd / 5,
                                "trials_per_solve": tdd / 5, "chi2_final": ld["chi2_final"]}
    sd.close()
    # the reference's live configuration with the reference Huber gate (gate_mode 0): survey-default
    # C3 seed 0 (free gauge, left image only, 2 % outliers; backend_lego.cpp:67-79, 92-94), timed
    # like value, with its own CPU baseline below and the oracle's reorder envelope as the parity check
    wl = make_window("C3", "default", args.seed, 0, 1)
    sl0 = lego_ba.Solver(device=local)
    sl0.upload(wl)
    sl0.solve_resident()
    nl0 = max(5, min(200, args.steps // 5))
    dl0, il0, tl0, ll0 = time_solves(sl0, nl0, barrier)
    out["live_config_c3"] = {"family": "default (survey)", "seed": args.seed, "gate_mode": 0,
                             "iterations_per_s": round(il0 / dl0, 3), "ms_per_solve": round(dl0 / nl0 * 1e3, 4),
                             "trials_per_s": round(tl0 / dl0, 3), "ms_per_trial": round(dl0 / tl0 * 1e3, 5),
                             "iterations_per_solve": il0 / nl0, "trials_per_solve": tl0 / nl0,
                             "chi2_final": ll0["chi2_final"], "solves": nl0}
    sl0.close()
    # the same window through the PCG reduced solve (BASELINE config 3 names "Schur + PCG"; the
    # reference's own solver, and value above, is the LDLT)
    sp = lego_ba.Solver(device=local, linear_solver=lego_ba.LH_SOLVER_PCG)
    sp.upload(w)
    sp.solve_resident()
    npcg = max(3, min(20, args.steps // 4))
    dp, ip, _, rp = time_solves(sp, npcg, barrier)
    out["pcg"] = {"ms_per_solve": round(dp / npcg * 1e3, 4), "iterations_per_s": round(ip / dp, 3),
                  "iterations_per_solve": ip / npcg, "pcg_steps_per_solve": rp["pcg_iterations"],
                  "chi2_rel_vs_ldlt": abs(rp["chi2_final"] - last["chi2_final"]) / last["chi2_final"]}
    sp.close()
    # the same window with lh_options.precision = FP32_RESID (BASELINE config 2's "fp32 residuals + fp64
    # accumulate"): k_lin's time and the solve's chi2 against the fp64 value line
    sf = lego_ba.Solver(device=local, precision=lego_ba.LH_PREC_FP32_RESID)
    sf.upload(w)
    sf.solve_resident()
    nf = max(3, min(20, args.steps // 4))
    df, itf, tf, rf = time_solves(sf, nf, barrier)
    out["fp32_resid"] = {"ms_per_solve": round(df / nf * 1e3, 4), "iterations_per_s": round(itf / df, 3),
                         "iterations_per_solve": itf / nf, "trials_per_solve": tf / nf,
                         "k_lin_ms": round(sf.time_lin_ms(reps=50), 5), "chi2_final": rf["chi2_final"],
                         "chi2_rel_vs_fp64": abs(rf["chi2_final"] - last["chi2_final"]) / last["chi2_final"]}
    sf.close()
    # a 64-keyframe window of C3's size (windows past 21 keyframes, the reduced
    # system of 384 rows: banded, k_ctrl_b), against the oracle's final chi2
    from windows import STABLE
    w64 = lego_ba.generate_window(P=64, L=50000, k=8, seed=args.seed, **dict(STABLE, outlier_frac=0.0))
    f64 = np.zeros(64, np.uint8)
    f64[0] = 1
    w64["pose_fixed"] = f64
    s64 = lego_ba.Solver(device=local)
    s64.upload(w64)
    ctl64 = s64.controller()
    s64.solve_resident()
    d64, i64, t64, l64 = time_solves(s64, 5, barrier)
    s64.set_profiling(True)
    s64.kernel_stats_reset()
    time_solves(s64, 2, barrier)
    k64 = s64.kernel_stats()
    s64.set_profiling(False)
    s64.close()
    out["p64_window"] = {"keyframes": 64, "landmarks": 50000, "obs": len(w64["obs_pose"]), "controller": ctl64,
                         "iterations_per_s": round(i64 / d64, 3), "ms_per_solve": round(d64 / 5 * 1e3, 3),
                         "iterations_per_solve": i64 / 5, "trials_per_solve": t64 / 5,
                         "controller_ms_per_trial": round(k64["k_ctrl"][1] / max(1, k64["k_ctrl"][0]), 4),
                         "kernels_ms_per_solve_event_bracketed": {k: round(v[1] / 2, 4) for k, v in k64.items()}}
    # the same 64 keyframes through the dense global-memory LDL^T (k_ctrl_g, LH_NO_BAND), the round-3 path
    os.environ["LH_NO_BAND"] = "1"
    sg = lego_ba.Solver(device=local)
    sg.upload(w64)
    os.environ.pop("LH_NO_BAND")
    sg.solve_resident()
    sg.set_profiling(True)
    sg.kernel_stats_reset()
    time_solves(sg, 2, barrier)
    kg = sg.kernel_stats()
    out["p64_window"]["dense_k_ctrl_g_ms_per_trial"] = round(kg["k_ctrl"][1] / max(1, kg["k_ctrl"][0]), 4)
    sg.close()
    # windows of 128 and 256 keyframes through the reference's LDL^T (banded, k_ctrl_b)
    for P_ in (128, 256):
        wb = lego_ba.generate_window(P=P_, L=50000, k=8, seed=3, **dict(STABLE, outlier_frac=0.0))
        fb_ = np.zeros(P_, np.uint8)
        fb_[0] = 1
        wb["pose_fixed"] = fb_
        sb = lego_ba.Solver(device=local)
        sb.upload(wb)
        sb.solve_resident()
        db, ib, tb, _ = time_solves(sb, 3, barrier)
        sb.set_profiling(True)
        sb.kernel_stats_reset()
        time_solves(sb, 1, barrier)
        kb = sb.kernel_stats()
        out[f"p{P_}_window_ldlt"] = {"keyframes": P_, "landmarks": 50000, "obs": len(wb["obs_pose"]),
                                     "controller": sb.controller(), "iterations_per_s": round(ib / db, 3),
                                     "ms_per_solve": round(db / 3 * 1e3, 3), "trials_per_solve": tb / 3,
                                     "controller_ms_per_trial": round(kb["k_ctrl"][1] / max(1, kb["k_ctrl"][0]), 4)}
        sb.set_profiling(False)
        sb.close()
    # a 128-keyframe window of C3's size through the PCG reduced solve (k_ctrl_p,
    # S p over the block-sparse pose-pair blocks), against the oracle's PCG below
    w128 = lego_ba.generate_window(P=128, L=50000, k=8, seed=3, **dict(STABLE, outlier_frac=0.0))
    f128 = np.zeros(128, np.uint8)
    f128[0] = 1
    w128["pose_fixed"] = f128
    s128 = lego_ba.Solver(device=local, linear_solver=lego_ba.LH_SOLVER_PCG)
    s128.upload(w128)
    s128.solve_resident()
    d128, i128, t128, l128 = time_solves(s128, 3, barrier)
    s128.set_profiling(True)
    s128.kernel_stats_reset()
    r128 = s128.solve_resident()
    k128 = s128.kernel_stats()
    s128.set_profiling(False)
    s128.close()
    out["p128_window_pcg"] = {"keyframes": 128, "landmarks": 50000, "obs": len(w128["obs_pose"]),
                              "iterations_per_s": round(i128 / d128, 3), "ms_per_solve": round(d128 / 3 * 1e3, 3),
                              "iterations_per_solve": i128 / 3, "trials_per_solve": t128 / 3,
                              "pcg_steps_per_trial": round(r128["pcg_iterations"] / max(1, r128["trials"]), 1),
                              "k_ctrl_p_ms_per_trial": round(k128["k_ctrl"][1] / max(1, k128["k_ctrl"][0]), 4),
                              "kernels_ms_per_solve_event_bracketed": {k: round(v[1], 4) for k, v in k128.items()}}
    # the frontend's pose-only LM (Frontend::EstimateCurrentPose): one frame the way
    # the reference calls it (frontend_lego.cpp:157, once per frame), and a batch of frames
    import frames
    sf = lego_ba.Solver(device=local)
    one = frames.batch(args.seed, 1, n_obs=150)
    sf.estimate_pose(one)
    lat, lat_dev = [], []
    for _ in range(20):
        t0 = time.perf_counter()
        r1 = sf.estimate_pose(one)
        lat.append((time.perf_counter() - t0) * 1e3)
        lat_dev.append(r1["time_ms"])
    nf = 2048
    fb = frames.batch(args.seed, nf, n_obs=150)
    sf.estimate_pose(fb)
    tms = [sf.estimate_pose(fb)["time_ms"] for _ in range(3)]
    out["estimate_pose"] = {"single_frame_ms": round(float(np.median(lat)), 4),
                            "single_frame_kernel_ms": round(float(np.median(lat_dev)), 4), "obs_per_frame": 150,
                            "batch_frames": nf, "batch_ms": round(min(tms), 4),
                            "batch_frames_per_s": round(nf / (min(tms) * 1e-3), 1),
                            "note": "single frame: host-to-host lh_estimate_pose call (4 rounds of solve(10)); "
                                    "batch: device time of one launch"}
    sf.close()
    # pyramidal LK optical flow (LKOpticalFlow4Layer): a KITTI-sized pair
    # (1241 x 376), 2000 keypoints, forward mode with an initial guess (the frontend's call)
    import images
    li1, li2 = images.pair(376, 1241, shift=(3.1, 0.4), seed=11)
    lk1 = images.keypoints(376, 1241, 2000, seed=11, border=False)
    lki = lk1 + np.float32([2.0, 0.0])
    sl = lego_ba.Solver(device=local)
    sl.lk_track(li1, li2, lk1, kp2_init=lki)
    lt = sorted(sl.lk_track(li1, li2, lk1, kp2_init=lki)["time_ms"] for _ in range(5))
    t0 = time.perf_counter()
    lr = sl.lk_track(li1, li2, lk1, kp2_init=lki)
    lh_ms = (time.perf_counter() - t0) * 1e3
    sl.close()
    out["lk_optical_flow"] = {"image": "1241x376 u8", "keypoints": len(lk1), "levels": 4,
                              "device_ms": round(lt[2], 4), "keypoints_per_s": round(len(lk1) / (lt[2] * 1e-3), 1),
                              "host_call_ms": round(lh_ms, 3), "tracked": int(lr["success"].sum()),
                              "note": "device_ms: pyramids of both images + tracking, median of 5; host_call_ms "
                                      "includes the image and keypoint copies"}
    if not args.no_cpu:
        import oracle_bind
        lib_path, flags = native_oracle()
        hi = host_info()
        threads = hi["cpus_usable"]
        o = oracle_bind.solve(w, n_threads=threads, lib_path=lib_path)   # warm-up
        t0 = time.perf_counter()
        its = nsolve = 0
        while True:
            o = oracle_bind.solve(w, n_threads=threads, lib_path=lib_path)
            its += o["iterations"]
            nsolve += 1
            ct = time.perf_counter() - t0
            if ct >= args.cpu_seconds:
                break
        out["cpu_baseline"] = {"value": round(its / ct, 4), "unit": "LM iterations/s", "cores": threads, "kind": "port",
                               "sample": f"{nsolve} full solve(10)s of the same C3 window by the block-sparse oracle "
                                         f"(oracle/lego_oracle.c ref_sparse, gcc {flags}, OpenMP {threads} threads = "
                                         f"every CPU this process may use: affinity mask capped by the cgroup "
                                         f"quota), {ct:.1f} s, {its} iterations",
                               "host": hi}
        out["chi2_rel_vs_oracle"] = abs(last["chi2_final"] - o["chi2_final"]) / o["chi2_final"]
        op = oracle_bind.solve(w, n_threads=threads)
        out["native_build_matches_parity_build"] = bool(op["chi2_final"] == o["chi2_final"])
        out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 2)
        od = oracle_bind.solve(wd, n_threads=threads, gate_mode=1, lib_path=lib_path)
        # live configuration: CPU baseline on the same window, and the oracle's own outcomes under
        # summation reorders (thread counts): the GPU's final chi2 must lie inside that envelope
        lc = out["live_config_c3"]
        env = [oracle_bind.solve(wl, n_threads=t, lib_path=lib_path) for t in sorted({1, 2, 8, threads})]
        t0 = time.perf_counter()
        its_l = ns_l = tr_l = 0
        while True:
            ol = oracle_bind.solve(wl, n_threads=threads, lib_path=lib_path)
            its_l += ol["iterations"]
            tr_l += ol["trials"]
            ns_l += 1
            ctl = time.perf_counter() - t0
            if ctl >= args.cpu_seconds / 2:
                break
        lo = min(r["chi2_final"] for r in env)
        hi = max(r["chi2_final"] for r in env)
        lc["cpu_baseline"] = {"value": round(its_l / ctl, 4), "unit": "LM iterations/s", "cores": threads, "kind": "port",
                              "trials_per_s": round(tr_l / ctl, 3),
                              "sample": f"{ns_l} full solve(10)s of this window by the block-sparse oracle, {ctl:.1f} s"}
        lc["speedup_vs_cpu"] = round(lc["iterations_per_s"] / lc["cpu_baseline"]["value"], 2)
        lc["speedup_vs_cpu_trials"] = round(lc["trials_per_s"] / lc["cpu_baseline"]["trials_per_s"], 2)
        lc["oracle_envelope"] = {"threads": sorted({1, 2, 8, threads}), "chi2_min": lo, "chi2_max": hi,
                                 "iterations": sorted({r["iterations"] for r in env}),
                                 "trials": sorted({r["trials"] for r in env})}
        lc["gpu_chi2_in_oracle_envelope"] = bool(lo * (1 - 1e-6) <= ll0["chi2_final"] <= hi * (1 + 1e-6))
        out["survey_default_c3"]["chi2_rel_vs_oracle"] = abs(ld["chi2_final"] - od["chi2_final"]) / od["chi2_final"]
        out["survey_default_c3"]["oracle_iterations"] = od["iterations"]
        t0 = time.perf_counter()
        o64 = oracle_bind.solve(w64, n_threads=threads, lib_path=lib_path)
        c64 = time.perf_counter() - t0
        out["p64_window"]["chi2_rel_vs_oracle"] = abs(l64["chi2_final"] - o64["chi2_final"]) / o64["chi2_final"]
        out["p64_window"]["oracle_iterations"] = o64["iterations"]
        out["p64_window"]["cpu_oracle_iterations_per_s"] = round(o64["iterations"] / c64, 3)
        out["p64_window"]["cpu_oracle_threads"] = threads
        t0 = time.perf_counter()
        o128 = oracle_bind.solve(w128, n_threads=threads, linear_solver=1, lib_path=lib_path)
        c128 = time.perf_counter() - t0
        pc = out["p128_window_pcg"]
        pc["chi2_rel_vs_oracle_pcg"] = abs(l128["chi2_final"] - o128["chi2_final"]) / o128["chi2_final"]
        pc["oracle_iterations"] = o128["iterations"]
        pc["cpu_oracle_iterations_per_s"] = round(o128["iterations"] / c128, 3)
        pc["cpu_oracle_threads"] = threads
        t0 = time.perf_counter()
        ol = oracle_bind.lk_track(li1, li2, lk1, kp2_init=lki, lib_path=lib_path)
        out["lk_optical_flow"]["cpu_oracle_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        out["lk_optical_flow"]["cpu_oracle_threads"] = 1
        out["lk_optical_flow"]["bitwise_equal_to_oracle"] = bool(np.array_equal(ol["kp2"], lr["kp2"]) and
                                                                  np.array_equal(ol["success"], lr["success"]))
        if lib_path:
            try:
                os.unlink(lib_path)
            except OSError:
                pass
    print(json.dumps(out))


if __name__ == "__main__":
    main()
