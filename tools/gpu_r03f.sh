# round 3: the COMPACT layer layout -- GPU parity of the layouts, then packed vs compact A/B on configs 3 and 5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tuples.py -m gpu > gpurun_out/r03f_tuples.log 2>&1 || { tail -30 gpurun_out/r03f_tuples.log; exit 1; }
tail -2 gpurun_out/r03f_tuples.log
AB_CASES=tile/packed,tile/compact timeout -k 10 400 python -u tools/ab_kernels.py 10000000 15 3 > gpurun_out/r03f_ab_cfg3.log 2>&1 || { tail -20 gpurun_out/r03f_ab_cfg3.log; exit 2; }
AB_ML=12 AB_CASES=po/packed,po/compact timeout -k 10 400 python -u tools/ab_kernels.py 10000000 15 5 > gpurun_out/r03f_ab_cfg5.log 2>&1 || { tail -20 gpurun_out/r03f_ab_cfg5.log; exit 3; }
grep -E "median" gpurun_out/r03f_ab_cfg3.log gpurun_out/r03f_ab_cfg5.log
