"""The oracle (CPU) on C4 stable_noout seed 0 at OpenMP thread counts 1-8, with the reference Huber gate
(gate_mode 0) and with its rounding residue taken as 0 (gate_mode 1): iterations, trials, final chi2 and
traces per summation order.  Output: profiles/r03_c4_oracle_gate_envelope.json."""
import sys, time, json
import os; R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, os.path.join(R, "lego-slam_amd", "python")); sys.path.insert(0, os.path.join(R, "tests")); os.chdir(R)
import numpy as np
import oracle_bind as ob
from windows import window
w = window("C4", seed=0, family="stable_noout")
res = {}
for gate in (0, 1):
    for t in (1, 2, 3, 4, 5, 6, 7, 8):
        t0 = time.time()
        o = ob.solve(w, n_threads=t, gate_mode=gate)
        res[f"g{gate}_t{t}"] = dict(it=o["iterations"], tr=o["trials"], acc=o["accepted"], chi=o["chi2_final"],
                                     trace=list(o["trace_chi2"]), lam=list(o["trace_lambda"]), sec=time.time()-t0)
        print(gate, t, o["iterations"], o["trials"], repr(o["chi2_final"]), f"{time.time()-t0:.1f}s", flush=True)
json.dump(res, open("profiles/r03_c4_oracle_gate_envelope.json", "w"))
