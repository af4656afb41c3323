"""Diagnostic: k_ctrl latency by phase (thread 0's wall clock at the barrier-aligned phase
boundaries) from the -DLH_STAMPS build: LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so.
The stamps' atomics perturb the kernel a little; shares and orders of magnitude only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lego-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lego_ba  # noqa: E402
from windows import window  # noqa: E402

NAMES = ["start", "prefetch + LM decision", "staged system arrived", "wave 0's scatter share", "block 0 factor + barrier", "unit words",
         "LDLT steps", "back substitution", "dx scatter", "trig / q_T", "pose compose", "pose / table stores", "tail"]
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
if cfg.startswith("P"):   # P<n>: an n-keyframe window of C3's size (n > 21: k_ctrl_g; its phase 5 is unused)
    from windows import STABLE
    import numpy as np
    P = int(cfg[1:])
    w = lego_ba.generate_window(P=P, L=50000, k=8, seed=0, **dict(STABLE, outlier_frac=0.0))
    w["pose_fixed"] = np.eye(1, P, dtype=np.uint8)[0]
else:
    w = window(cfg, seed=0, family="stable_noout")
s = lego_ba.Solver(device=0)
s.upload(w)
s.solve_resident()
lego_ba.debug_stamps(reset=True)
for _ in range(5):
    s.solve_resident()
st = [int(x) for x in lego_ba.debug_stamps(reset=True)]
n = st[61]
cyc = [st[32 + i] for i in range(len(NAMES))]
tot_cyc = (cyc[-1] - cyc[0]) / n
tot_ns = (st[63] - st[62]) / n * 10.0
print(f"{cfg}: {n} live k_ctrl launches, {tot_cyc:.0f} cycles = {tot_ns / 1000:.2f} us start-to-end "
      f"(clock {tot_cyc / tot_ns:.2f} GHz)")
prev = 0
for i in range(1, len(NAMES)):
    if cyc[i] == 0:   # a phase this build does not stamp (round 4: no pivot rank, no separate commit)
        continue
    d = (cyc[i] - cyc[prev]) / n
    prev = i
    print(f"  {NAMES[i]:22s} {d:9.0f} cycles {d / tot_cyc * 100:5.1f}%  {d / (tot_cyc / tot_ns) / 1000:6.2f} us")
if cfg.startswith("P"):   # k_ctrl_g's panel sub-phases, summed over the panels: (a) load, (b) diagonal
    # block, (c) rows below, (d)+(e) write-back and trailing tiles (stamps 13-16 follow stamp 5)
    sub = [st[32 + 5]] + [st[32 + i] for i in (13, 14, 15, 16)]
    for nm, i in (("(a) panel load", 1), ("(b) diagonal block", 2), ("(c) rows below", 3), ("(d)+(e) trailing", 4)):
        k = st[32 + 13] and n
        d = (sub[i] - sub[i - 1]) / n if i > 1 else None
        if d is not None:
            print(f"    {nm:20s} {d:9.0f} cycles  {d / (tot_cyc / tot_ns) / 1000:6.2f} us")
# per-step split of the LDL^T loop (lds_ldlt_solve stamps 46-51): wave 0's diagonal tile, its 8x8
# factor, its wait at the step barrier; the other 15 waves' unit time and barrier wait (per wave)
nl = max(st[51], 1)
if st[51]:
    print(f"  LDLT loop per launch: wave 0 diag tile {st[46] / nl:.0f}, factor {st[47] / nl:.0f}, barrier wait "
          f"{st[48] / nl:.0f} cycles; other waves (mean per wave) unit {st[49] / nl / 15:.0f}, barrier wait "
          f"{st[50] / nl / 15:.0f} cycles")
# per step t of the LDL^T loop (stamps 64-127): wave 0's diagonal tile, factor and barrier wait (mean
# per launch) and the slowest other wave's unit (the worst launch)
if len(st) >= 128 and st[51]:
    # the worst unit's stamp: cycles << 24 | its unit word << 4 | its wave
    print("  step  w0 tile  w0 factor  w0 wait  worst unit  (wave: tile row I, tile columns [j0, j1), S = stores L)")
    for t in range(16):
        a, b, c, m = st[64 + t] / nl, st[80 + t] / nl, st[96 + t] / nl, st[112 + t]
        if a or b or c or m:
            cyc, uw, wv = m >> 24, (m >> 4) & 0xffff, m & 15
            desc = f"w{wv}: I+{uw & 7} [{(uw >> 3) & 7}, {(uw >> 6) & 15}){' S' if uw & 0x4000 else ''}" if uw & 0x8000 else ""
            print(f"  {t:4d} {a:8.0f} {b:10.0f} {c:8.0f} {cyc:11d}  {desc}")
# the waves' SIMDs (stamps 160-175: HW_ID, SIMD_ID in bits 5:4, bit 32 set once written)
if len(st) >= 176 and any(st[160 + w] >> 32 for w in range(16)):
    print("  wave -> SIMD: " + " ".join(f"{w}:{(st[160 + w] >> 4) & 3}" for w in range(16) if st[160 + w] >> 32))
# k_ctrl_b's back substitution (stamps 52-55): per block, wave 0's x_b = ND_b y_b (ND read, broadcasts, dot)
# and its row updates (readlanes, dots, the entering row), and its ring readiness checks
if st[55]:
    nb_ = st[55]
    print(f"  back substitution per block: x_b {st[52] / nb_:.0f}, row updates {st[53] / nb_:.0f}, "
          f"ring checks {st[54] / nb_:.0f} cycles ({nb_ // max(n, 1)} blocks per launch)")
# k_ctrl_b's loader wave 12 at the tile-row writes (stamps 56-58): the wait for its value loads, the writes
if st[58]:
    print(f"  loader per tile row: value-load wait {st[56] / st[58]:.0f}, window writes {st[57] / st[58]:.0f} cycles")
# k_ctrl_b's barrier arrival per wave (stamps 128-159), mean per step, even and odd steps
if len(st) >= 160 and any(st[128:160]):
    ns = max(nl, 1) * 48   # 96 steps per launch at P = 128: an approximate per-step mean
    for par, nm in ((0, "even"), (1, "odd")):
        print(f"  barrier arrival, {nm} steps (sum over launches / launches / half the steps, per wave):",
              " ".join(f"{st[128 + 16 * par + w] / max(n, 1) / max(1, (st[51] and 48)):.0f}" for w in range(16)))
