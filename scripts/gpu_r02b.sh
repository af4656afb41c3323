# GPU tests, then the PMC passes of the bench (scripts/gpu_pmc.sh); stops at the first failure.
set -u
bash scripts/gpu_r02.sh tests || exit $?
bash scripts/gpu_pmc.sh
