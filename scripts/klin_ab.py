"""k_lin variants (library builds under lego-slam_amd/lib/ab/<name>/) against the current library: the
C3 k_lin launch time and solve by chunk size (scripts/chunk_sweep.py), each build in a fresh process, and
the single-trial / bitwise / stable-window parity tests on each variant.
usage: python3 scripts/klin_ab.py NAME[:CHUNKS] ...   (CHUNKS: '-'-separated chunk sizes, default 0)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "lego-slam_amd", "lib")
arms = [("current", os.path.join(LIB, "liblego_ba.so"), ["0"])]
for a in sys.argv[1:]:
    name, _, ch = a.partition(":")
    arms.append((name, os.path.join(LIB, "ab", name, "liblego_ba.so"), (ch or "0").split("-")))
for rnd in range(2):
    for name, lib, ch in arms:
        env = dict(os.environ, LH_LIB=lib)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "chunk_sweep.py")] + ch, env=env,
                           capture_output=True, text=True, timeout=300)
        for ln in (r.stdout + r.stderr).strip().splitlines()[-len(ch) - 2:]:
            print(rnd, name, ln, flush=True)
for name, lib, ch in arms[1:]:
    env = dict(os.environ, LH_LIB=lib)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "--timeout", "120", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_parity.py"), "-k",
                        "single_trial or bitwise or parity_stable or c3_window or strategy1_single"],
                       env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    print(name, "parity:", (r.stdout + r.stderr).strip().splitlines()[-1], flush=True)
