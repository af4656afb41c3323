# solve throughput vs the number of trials kept enqueued ahead of the device (lh_options.trials_per_sync)
set -o pipefail
mkdir -p gpurun_out/depth
for d in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 500 --warmup 3 --no-cpu --no-extras --trials-per-sync $d > gpurun_out/depth/d$d.json 2> gpurun_out/depth/d$d.err || exit 1
done
