"""Diagnostic: k_frames per-phase wave-cycles per LM trial on single frames (the -DLH_STAMPS build:
LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so).  Phases 0-2 are summed over the four waves, 3-4 and
6-7 are wave 0 only, 5 is the end-of-trial barrier (all waves)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lego-slam_amd", "python"), os.path.join(ROOT, "tests")]
import lego_ba  # noqa: E402
import frames   # noqa: E402

s = lego_ba.Solver()
one = frames.batch(0, 1, n_obs=150)
s.estimate_pose(one)
lego_ba.debug_stamps(reset=True)
N = 20
its = 0
for _ in range(N):
    r = s.estimate_pose(one)
    its += int(r["iterations"][0])
st = [int(x) for x in lego_ba.debug_stamps(reset=True)]
names = ["edge work (4 waves)", "rows + column sums (4 waves)", "barrier after sums (4 waves)",
         "wave 0: sums + LM decision", "wave 0: candidate pose", "end-of-trial barrier (4 waves)",
         "wave 0: system loads", "wave 0: 6x6 LDLT solve"]
print(f"{N} single-frame calls, {its / N:.1f} LM iterations per call (trials are at least that)")
for k, nm in enumerate(names):
    print(f"  {nm:32s} {st[24 + k] / N:12.0f} wave-cycles per call")
s.close()
