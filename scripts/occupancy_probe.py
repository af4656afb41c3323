"""k_lin's latency hiding, probed: the C3 trial-mode k_lin (lh_debug_time_lin, 50 back-to-back replays) at its
normal two workgroups per CU (104 landmarks per chunk, ~488 chunks) against one workgroup per CU: 208 landmarks per
chunk (~244 chunks, one per CU), also with 24 KB of extra LDS per workgroup (LH_TEST_LIN_LDS_PAD: two no longer
fit a CU), and 104 per chunk with the pad (two rounds of chunks).  The same
work at half the waves per SIMD: how much the second wave hides bounds what a third could."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys
sys.path[:0] = [%r, %r]
import lego_ba
from windows import window
w = window("C3", seed=0, family="stable_noout")
s = lego_ba.Solver(chunk_landmarks=int(sys.argv[1]))
s.upload(w)
s.solve_resident()
ms = sorted(s.time_lin_ms(50) for _ in range(5))[2]
print(f"chunk_landmarks {sys.argv[1]} lds_pad {sys.argv[2]}: k_lin {1e3 * ms:.2f} us")
""" % (os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python"))
for clm, pad in ((0, 0), (208, 0), (208, 24000), (104, 24000)):
    env = dict(os.environ)
    if pad:
        env["LH_TEST_LIN_LDS_PAD"] = str(pad)
    r = subprocess.run([sys.executable, "-c", CHILD, str(clm), str(pad)], env=env, capture_output=True, text=True,
                       timeout=300)
    print(r.stdout.strip() or r.stderr[-500:], flush=True)
