# PMC passes over the bench (separate runs; counters only with --kernel-trace, never with sys/runtime traces)
set -u
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, counters...
    local nm=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc/$nm -o $nm --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/pmc/$nm.log 2>&1
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS || exit $?
run sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_BUSY_CYCLES || exit $?
run fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
run write WRITE_SIZE || exit $?
