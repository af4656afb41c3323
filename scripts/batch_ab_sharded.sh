# The N = 2 bench line (C4 sharded two ways) rehearsed on one GPU over the one-shot peer-write exchange, with batched
# rejection runs and without (LH_NO_BATCH=1), alternated twice: the relative cost of a sharded solve's rejection
# chains (the ranks share the GPU, so the absolute times say nothing about two GPUs).  usage: TAG=x bash scripts/batch_ab_sharded.sh
set -u
OUT=gpurun_out/${TAG:-batch_sharded}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rnd in 1 2; do
    for mode in batch serial; do
        if [ $mode = serial ]; then export LH_NO_BATCH=1; else unset LH_NO_BATCH; fi
        timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
            --master-port 29503 bench.py --gpus 2 --steps 20 --warmup 2 --comm p2p --no-cpu --no-extras \
            > "$OUT/n2_${mode}_$rnd.json" 2> "$OUT/n2_${mode}_$rnd.err" || { tail -20 "$OUT/n2_${mode}_$rnd.err"; exit 1; }
        python3 -c "
import json; d = json.loads(open('$OUT/n2_${mode}_$rnd.json').read().strip().splitlines()[-1])
print('$mode $rnd', d['value'], 'ms/solve', d['ms_per_step'], 'trials', d['trials_per_solve'], 'iters', d['iterations_per_solve'])"
    done
done
