# diagnostic: lds_ldlt_solve in isolation (lego-slam_amd/tools/ubench_ldlt*.hip)
set -u
mkdir -p gpurun_out
B=lego-slam_amd/lib
{
for b in ubench_ldlt_old ubench_ldlt ubench_ldlt_st; do
  [ -x $B/$b ] || continue
  echo "== $b"; for n in ${NS:-120 42 6}; do timeout -k 5 60 $B/$b $n || exit 1; done
done
for b in ubench_ldlt_parts exp_ldlt; do
  if [ -x $B/$b ]; then echo "== $b"; timeout -k 5 60 $B/$b || exit 1; fi
done
} > gpurun_out/u.log 2>&1
if [ "${RUN_TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -m pytest tests -q -m gpu -rf -p no:cacheprovider -k "${TESTS_K:-reduced_solve or parity_stable or p21 or subsets}" > gpurun_out/t.log 2>&1; rc=$?; echo rc=$rc >> gpurun_out/t.log
exit $rc
fi
