# round 3 (re-entry): the restored tree on a fresh box -- the whole -m gpu suite, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03g_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03g_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03g_gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03g_bench_cfg3.json 2> gpurun_out/r03g_bench_cfg3.err || { tail -20 gpurun_out/r03g_bench_cfg3.err; exit 2; }
head -c 1500 gpurun_out/r03g_bench_cfg3.json
echo
timeout -k 10 300 python -u tools/ab_cfg2.py 1000000 60 > gpurun_out/r03g_ab_cfg2.log 2>&1 || { tail -20 gpurun_out/r03g_ab_cfg2.log; exit 3; }
cat gpurun_out/r03g_ab_cfg2.log
tools/sq_counters.sh r03g 2 || exit 4
AB_CASES=tile/packed,tile/packed-win3,tile/packed-win3x1k timeout -k 10 400 python -u tools/ab_kernels.py 10000000 15 3 > gpurun_out/r03g_ab_win3.log 2>&1 || { tail -20 gpurun_out/r03g_ab_win3.log; exit 5; }
grep -E "median|identical" gpurun_out/r03g_ab_win3.log
