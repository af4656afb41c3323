"""Per-launch HBM traffic of k_lin from the rocprofv3 PMC passes of scripts/gpu_pmc.sh.

MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB per dispatch;
on gfx950 FETCH_SIZE reports half of the bytes of wide (16 B/lane) coalesced reads, so it
is doubled; WRITE_SIZE is exact for 16 B/lane stores.  k_lin's reads are the 16-B landmark
records and observation words (mixed 16/8/4 B per lane: the doubling is an upper bound for
the narrow part).  Writes a JSON for bench.py's roofline.traffic.
usage: python scripts/pmc_traffic.py gpurun_out/pmc profiles/r01_pmc_k_lin.json P20-L50000-k8-stable_noout-s0
"""
import csv
import glob
import json
import sys
from collections import defaultdict

root, out_path, workload = sys.argv[1], sys.argv[2], sys.argv[3]
kern = "k_lin<3, true, false>"
vals = defaultdict(list)
for f in glob.glob(f"{root}/*/*_counter_collection.csv"):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("void " + kern) or r["Kernel_Name"].startswith(kern):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    active = {d for (d, c), v in per.items() if c in ("FETCH_SIZE", "WRITE_SIZE") and v > 1024.0}
    for (d, c), v in per.items():
        if d in active:          # early-exit launches after the stop flag carry no traffic
            vals[c].append(v)
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
res = {"workload": workload, "kernel": kern, "dispatches": len(vals["FETCH_SIZE"]),
       "FETCH_SIZE_KiB": round(fetch, 1), "WRITE_SIZE_KiB": round(write, 1),
       "bytes_per_launch": int(2 * fetch * 1024 + write * 1024),
       "correction": "2 x FETCH_SIZE (gfx950 wide-read half count) + WRITE_SIZE"}
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps(res))
