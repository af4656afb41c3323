"""The drop-in call from the compiled C++ caller (tests/abi_caller.cpp: lh_solve on host buffers, median of 15) for
two builds on one box, alternated three times: the current lego-slam_amd/lib/abi_caller against the caller and
library in the directory given (an older tree's build; its rpath loads the library beside it)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import bench  # noqa: E402

other = sys.argv[1]
w = bench.make_window("C3", "stable_noout", 0, 0, 1)
for rep in range(3):
    for name, exe in (("current", None), (other, os.path.join(other, "abi_caller"))):
        line = bench.cxx_caller_ms(w, 15, exe=exe, line=True)
        print(rep, name, line, flush=True)
