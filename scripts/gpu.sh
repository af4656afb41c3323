# One parameterised driver for every GPU call (gpurun):  bash scripts/gpu.sh STEP [STEP ...]
# Each step runs under its own time limit and writes under gpurun_out/<tag>/; the first failing step
# ends the call (no further GPU work after a fault, an abort or a timeout).  TAG (default "run") names
# the output directory, so one call's evidence can be copied to profiles/ as a unit.
#
#   tests[=FILES]      pytest -m gpu on FILES (default: tests/), verbose, per-test timeout
#   smoke              __graft_entry__.smoke()
#   bench[=ARGS]       bench.py ARGS (default: the contract's default run, CPU baseline included)
#   quick              bench.py --steps 200 --warmup 3 --no-cpu --no-extras
#   trace              rocprofv3 --kernel-trace --stats of the quick bench (per-kernel averages)
#   pmc                the PMC passes over the quick bench (one counter group per run)
#   stamps=CFG         k_ctrl phase stamps (diagnostic -DLH_STAMPS library) on window CFG (C3, P64, ...)
#   linstamps=CFG      k_lin / k_reduce per-phase wave-cycle shares (the same diagnostic library)
#   ab=LIB             rocprofv3 A/B of the current library against LIB, alternated twice (k_lin, k_reduce,
#                      k_ctrl* averages and the bench line of each)
#   py=SCRIPT[,ARGS]   python3 SCRIPT ARGS (a measurement script under scripts/)
#   pytrace=SCRIPT[,ARGS]  rocprofv3 --kernel-trace --stats of that script (per-kernel averages; the raw trace kept)
#   bin=PATH           a diagnostic binary built in-tree (lego-slam_amd/lib/ubench_*)
#   env=VAR=VALUE      export VAR for the steps after it (their outputs get a _VAR_VALUE suffix); unenv=VAR
set -u
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
QUICK="bench.py --steps 200 --warmup 3 --no-cpu --no-extras"
SFX=""

kstats() {   # label, rocprof output dir -> one summary line per kernel of interest
    for f in $(find "$2" -name '*kernel_stats.csv'); do
        python3 - "$1" "$f" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[2])):
    n = row.get("Name", "")
    if any(k in n for k in ("k_ctrl", "k_lin<", "k_reduce", "k_dense", "k_frames", "k_lk")):
        print(sys.argv[1], n[:28], row.get("Calls"), row.get("AverageNs"))
PY
    done
}

for step in "$@"; do
    name=${step%%=*}
    arg=""
    [ "$name" != "$step" ] && arg=${step#*=}
    echo "== $step" >> "$OUT/steps.log"
    case $name in
    tests)
        arg=${arg:-tests}
        timeout -k 10 900 python -u -m pytest ${arg//,/ } -m gpu -x -v -rf --timeout 300 --timeout-method thread \
            -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
        tail -1 "$OUT/tests.log" ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
        cat "$OUT/smoke.log" ;;
    bench)
        timeout -k 10 600 python3 bench.py $arg > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
        tail -c 600 "$OUT/bench.json" ;;
    quick)
        timeout -k 10 300 python3 $QUICK > "$OUT/quick$SFX.json" 2> "$OUT/quick$SFX.err" || { tail -20 "$OUT/quick$SFX.err"; exit 1; }
        cat "$OUT/quick$SFX.json" ;;
    trace)
        rm -rf "$OUT/trace$SFX"
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace$SFX" -o run --output-format csv -- python3 $QUICK \
            > "$OUT/trace$SFX.log" 2>&1 || { tail -20 "$OUT/trace$SFX.log"; exit 1; }
        kstats "trace$SFX" "$OUT/trace$SFX" | tee "$OUT/trace_summary$SFX.txt" ;;
    pmc)
        mkdir -p "$OUT/pmc"
        pass() {   # name, counters...
            local nm=$1; shift
            timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/pmc/$nm" -o $nm --output-format csv -- \
                python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras > "$OUT/pmc/$nm.log" 2>&1
        }
        pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
        pass sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_BUSY_CYCLES || exit 1
        pass fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit 1
        pass write WRITE_SIZE || exit 1 ;;
    stamps)
        LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python3 scripts/ctrl_stamps.py ${arg:-C3} \
            > "$OUT/stamps_${arg:-C3}$SFX.log" 2>&1 || { cat "$OUT/stamps_${arg:-C3}$SFX.log"; exit 1; }
        cat "$OUT/stamps_${arg:-C3}$SFX.log" ;;
    linstamps)
        LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python3 scripts/stamps.py ${arg:-C3} \
            > "$OUT/linstamps_${arg:-C3}.log" 2>&1 || { cat "$OUT/linstamps_${arg:-C3}.log"; exit 1; }
        cat "$OUT/linstamps_${arg:-C3}.log" ;;
    ab)
        : > "$OUT/ab_summary.txt"
        for r in 1 2; do
            for v in A B; do
                lib=$( [ $v = A ] && echo lego-slam_amd/lib/liblego_ba.so || echo "$arg" )
                LH_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ab_$v$r" -o p --output-format csv -- \
                    python3 $QUICK > "$OUT/ab_bench_$v$r.json" 2> "$OUT/ab_bench_$v$r.err" || exit 1
                kstats "$v$r" "$OUT/ab_$v$r" >> "$OUT/ab_summary.txt"
                echo "$v$r $(cat "$OUT/ab_bench_$v$r.json")" | cut -c1-200 >> "$OUT/ab_summary.txt"
                rm -rf "$OUT/ab_$v$r"
            done
        done
        cat "$OUT/ab_summary.txt" ;;
    py)
        scr=${arg%%,*}
        rest=""
        [ "$scr" != "$arg" ] && rest=${arg#*,}
        timeout -k 10 600 python3 $scr ${rest//,/ } > "$OUT/$(basename $scr .py)$SFX.log" 2>&1 || { tail -30 "$OUT/$(basename $scr .py)$SFX.log"; exit 1; }
        tail -30 "$OUT/$(basename $scr .py)$SFX.log" ;;
    pytrace)
        scr=${arg%%,*}
        rest=""
        [ "$scr" != "$arg" ] && rest=${arg#*,}
        nm=pytrace_$(basename $scr .py)$SFX
        rm -rf "$OUT/$nm"
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/$nm" -o run --output-format csv -- python3 $scr ${rest//,/ } \
            > "$OUT/$nm.log" 2>&1 || { tail -20 "$OUT/$nm.log"; exit 1; }
        tail -8 "$OUT/$nm.log"
        kstats "$nm" "$OUT/$nm" | tee "$OUT/${nm}_summary.txt" ;;
    env)
        export "$arg"
        SFX="_${arg//[^A-Za-z0-9]/_}" ;;
    unenv)
        unset "$arg"
        SFX="" ;;
    bin)
        timeout -k 10 120 "$arg" > "$OUT/$(basename $arg).log" 2>&1 || { tail -30 "$OUT/$(basename $arg).log"; exit 1; }
        cat "$OUT/$(basename $arg).log" ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
