# The N > 1 bench path rehearsed on one GPU: N ranks over the host transport (gloo), each with its landmark
# shard of C4 (the N > 1 default), then the N = 1 line; one JSON line each under gpurun_out/$TAG/.  The ranks
# share one GPU and exchange through the host, so the times say nothing about N GPUs: this checks the line's
# definition and the multi-rank flow.  usage: TAG=x bash scripts/scale_rehearsal.sh
set -u
OUT=gpurun_out/${TAG:-scale}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --steps 100 --warmup 2 --no-cpu --no-extras > "$OUT/n1.json" 2> "$OUT/n1.err" || { tail -20 "$OUT/n1.err"; exit 1; }
for comm in host p2p; do
    timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29502 bench.py --gpus 2 --steps 10 --warmup 1 --comm $comm \
        > "$OUT/n2_$comm.json" 2> "$OUT/n2_$comm.err" || { tail -20 "$OUT/n2_$comm.err"; exit 1; }
done
for n in 1 2_host 2_p2p; do python3 -c "
import json; d = json.loads(open('$OUT/n$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['scaling'], d['config']['workload'], d['iterations_per_solve'], d['trials_per_solve'], d['ms_per_step'],
      d.get('c4_speedup_vs_1gpu'), d['config']['exchange'])"; done
