# The host C/C++ of the CPU path under sanitizers: the window planner with its worker pool
# (liblego_plan.so, lh_plan.cpp / lh_plan.h), the synthetic-window generator and the oracle, built with
# -fsanitize=thread and with -fsanitize=address,undefined (make san), then tests/test_plan_cpu.py,
# tests/test_window_gen.py and tests/test_oracle.py run against those builds (the sanitizer runtime preloaded
# into the interpreter; LH_PLAN_LIB / LH_WIN_LIB / LH_ORACLE_LIB select the builds).  The oracle's threads are
# OpenMP, whose runtime (libgomp) is not instrumented: its multi-threaded solves hang under TSan (the first one,
# test_stable_family_reproducible, did not finish in 15 minutes), so the oracle runs under ASan + UBSan only.  Logs: $OUT (default
# profiles/r06_sanitizers).  Exit status: nonzero if any run reported an error.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-profiles/r06_sanitizers}
mkdir -p "$OUT"
make -s -C lego-slam_amd san && make -s -C oracle san || exit 1
rc=0
for san in tsan asan; do
    TESTS="tests/test_plan_cpu.py tests/test_window_gen.py"
    [ $san = asan ] && TESTS="$TESTS tests/test_oracle.py"
    lib=$(gcc -print-file-name=lib$san.so)
    export LH_PLAN_LIB=lego-slam_amd/lib/san/$san/liblego_plan.so LH_WIN_LIB=lego-slam_amd/lib/san/$san/liblego_window.so
    export LH_ORACLE_LIB=oracle/_san/$san/liblego_oracle.so
    # tsan: reports fail the run (exitcode 66); the interpreter and libgomp are not instrumented
    # asan: leaks are the interpreter's (not checked); undefined behaviour aborts (-fno-sanitize-recover)
    TSAN_OPTIONS="exitcode=66 ignore_noninstrumented_modules=1 second_deadlock_stack=1" \
    ASAN_OPTIONS="detect_leaks=0 abort_on_error=1" UBSAN_OPTIONS="print_stacktrace=1" \
    LD_PRELOAD=$lib timeout -k 10 1800 python3 -m pytest $TESTS -q -s -m "not gpu" -p no:cacheprovider \
        > "$OUT/$san.log" 2>&1
    r=$?
    n=$(grep -c "WARNING: ThreadSanitizer\|ERROR: AddressSanitizer\|runtime error:" "$OUT/$san.log")
    echo "$san: pytest exit $r, sanitizer reports $n ($(tail -1 "$OUT/$san.log"))" | tee -a "$OUT/summary.txt"
    [ $r -ne 0 ] || [ "$n" -ne 0 ] && rc=1
done
exit $rc
