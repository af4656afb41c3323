"""Summarise hipcc's -Rpass-analysis=kernel-resource-usage remarks for lh_kernels.hip and fail
(exit 1) if any kernel uses scratch (a register spill): DESIGN.md states every solver kernel is
spill-free, and the Makefile runs this on every build.

usage: python3 scripts/resource_check.py lego-slam_amd/lib/lh_kernels.resource.txt [lh_lk.resource.txt ...]
"""
import re
import subprocess
import sys


def demangle(name):
    try:
        out = subprocess.run(["c++filt", name], capture_output=True, text=True, timeout=10).stdout.strip()
        return out.split("(")[0] or name
    except (OSError, subprocess.SubprocessError):
        return name


def parse(path):
    kernels, cur = [], None
    pat = re.compile(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                     r"LDS Size \[bytes/block\]):\s*(\S+)")
    with open(path) as f:
        for line in f:
            m = pat.search(line)
            if not m:
                continue
            key, val = m.group(1), m.group(2)
            if key == "Function Name":
                cur = {"name": demangle(val)}
                kernels.append(cur)
            elif cur is not None:
                cur[key.split(" ")[0]] = int(val)
    return kernels


# No kernel may spill (round 4: k_ctrl_g's rows-below loop addresses its LDS operands off one base
# register instead of ~160 constant-address VGPRs, which had pushed it 3 registers over its budget).
SPILL_ALLOWED = {}


def main():
    kernels = [k for path in sys.argv[1:] for k in parse(path)]
    if not kernels:
        print("resource_check: no kernel-resource-usage remarks found", file=sys.stderr)
        return 1
    bad = []
    print(f"{'kernel':<28} {'VGPR':>5} {'AGPR':>5} {'scratch':>8} {'waves/SIMD':>10} {'LDS B':>8}")
    for k in kernels:
        print(f"{k['name']:<28} {k.get('VGPRs', 0):>5} {k.get('AGPRs', 0):>5} {k.get('ScratchSize', 0):>8} "
              f"{k.get('Occupancy', 0):>10} {k.get('LDS', 0):>8}")
        if k.get("ScratchSize", 0) > SPILL_ALLOWED.get(k["name"], 0):
            bad.append(k["name"])
    if bad:
        print("resource_check: scratch (register spill) in " + ", ".join(bad), file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
