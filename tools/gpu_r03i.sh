# round 3: single-round 96-B / 80-B parse-only windows at higher occupancy -- A/B on config 4 (IMIX) and config 5
set -o pipefail
mkdir -p gpurun_out
AB_ML=0 AB_CASES=po/product,po/c6,po/c6w6,po/c5w6 timeout -k 10 400 python -u tools/ab_kernels.py 12500000 20 4 > gpurun_out/r03i_ab_cfg4.log 2>&1 || { tail -20 gpurun_out/r03i_ab_cfg4.log; exit 4; }
grep -E "median|identical" gpurun_out/r03i_ab_cfg4.log
AB_ML=12 AB_CASES=po/product,po/c6 timeout -k 10 400 python -u tools/ab_kernels.py 10000000 10 5 > gpurun_out/r03i_ab_cfg5.log 2>&1 || { tail -20 gpurun_out/r03i_ab_cfg5.log; exit 5; }
grep -E "median|identical" gpurun_out/r03i_ab_cfg5.log
