# round 3: cached (not non-temporal) record stores in the parse-only instances -- A/B on configs 5 and 4
set -o pipefail
mkdir -p gpurun_out
AB_ML=12 AB_CASES=po/packed,po/packed-cached timeout -k 10 400 python -u tools/ab_kernels.py 10000000 15 5 > gpurun_out/r03x_ab_cfg5.log 2>&1 || { tail -20 gpurun_out/r03x_ab_cfg5.log; exit 1; }
grep -E "median|identical" gpurun_out/r03x_ab_cfg5.log
AB_ML=0 AB_CASES=po/c6,po/c6-cached timeout -k 10 400 python -u tools/ab_kernels.py 12500000 15 4 > gpurun_out/r03x_ab_cfg4.log 2>&1 || { tail -20 gpurun_out/r03x_ab_cfg4.log; exit 2; }
grep -E "median|identical" gpurun_out/r03x_ab_cfg4.log
