# A/B of the k_lin chunk size (landmarks per workgroup) on C3: one bench line per setting.
set -u
mkdir -p gpurun_out/ab_chunk
for c in ${CHUNKS:-128 96 104 112 64 160}; do
    LH_CHUNK_LM=$c timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab_chunk/c$c.log 2>&1
    rc=$?; echo "rc=$rc" >> gpurun_out/ab_chunk/c$c.log
    [ $rc -eq 0 ] || exit $rc
done
