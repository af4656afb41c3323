"""A/B of the drop-in call (lh_solve on host buffers) between library builds, each in a fresh process
through the compiled C++ caller: python3 scripts/host_ab.py DIR [DIR ...], DIR holding abi_caller and its
liblego_ba.so ($ORIGIN rpath).  Alternates the builds three times; also the current build unpinned
(LH_HOST_PIN=0) and with the planner on 1 thread."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import bench  # noqa: E402

w = bench.make_window("C3", "stable_noout", 0, 0, 1)
cur = os.path.join(ROOT, "lego-slam_amd", "lib", "abi_caller")
arms = [("current", cur, None), ("current LH_HOST_PIN=0", cur, {"LH_HOST_PIN": "0"})]
arms += [(d, os.path.join(d, "abi_caller"), None) for d in sys.argv[1:]]
for r in range(3):
    for name, exe, env in arms:
        print(r, name, bench.cxx_caller_ms(w, 30, exe=exe, line=True, env=env), flush=True)
