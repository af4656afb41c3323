"""Diagnostic: 30 calls of the k_ctrl LDL^T probe on one random n = 120 SPD system (for a rocprofv3
kernel trace of k_ldlt_probe), and the solution's residual."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lego-slam_amd", "python"))
import numpy as np  # noqa: E402
import torch        # noqa: E402
import lego_ba      # noqa: E402

rng = np.random.default_rng(0)
n = 120
M = rng.standard_normal((n, n))
S = M @ M.T + n * np.eye(n)
b = rng.standard_normal(n)
lib = lego_ba.ba_lib()
lib.lh_debug_ldlt_probe.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
St = torch.tensor(S, dtype=torch.float64, device="cuda").contiguous()
bt = torch.tensor(b, dtype=torch.float64, device="cuda")
xt = torch.zeros(n, dtype=torch.float64, device="cuda")
for _ in range(30):
    assert lib.lh_debug_ldlt_probe(St.data_ptr(), bt.data_ptr(), n, xt.data_ptr()) == 0
x = xt.cpu().numpy()
print("residual", float(np.abs(S @ x - b).max()), flush=True)
