# a 2- and 4-rank rehearsal of the C4 scaling flow on one GPU (host transport), each under its own limit
set -u
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 3 --warmup 1 --comm host > gpurun_out/b_rehearse_$n.log 2>&1 || exit $?
done
