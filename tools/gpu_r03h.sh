# round 3: persistent parse-only kernel (next tile's descriptors + first-round window prefetched) -- A/B on configs 2, 4, 5
set -o pipefail
mkdir -p gpurun_out
AB_VARIANTS=0,63,70,71,73 timeout -k 10 300 python -u tools/ab_cfg2.py 1000000 60 > gpurun_out/r03h_ab_cfg2.log 2>&1 || { tail -20 gpurun_out/r03h_ab_cfg2.log; exit 3; }
cat gpurun_out/r03h_ab_cfg2.log
AB_ML=0 AB_CASES=po/product,po/persist,po/persist-c6,po/persist-half timeout -k 10 400 python -u tools/ab_kernels.py 12500000 15 4 > gpurun_out/r03h_ab_cfg4.log 2>&1 || { tail -20 gpurun_out/r03h_ab_cfg4.log; exit 4; }
grep -E "median|identical" gpurun_out/r03h_ab_cfg4.log
AB_ML=12 AB_CASES=po/packed,po/persist-packed timeout -k 10 400 python -u tools/ab_kernels.py 10000000 15 5 > gpurun_out/r03h_ab_cfg5.log 2>&1 || { tail -20 gpurun_out/r03h_ab_cfg5.log; exit 5; }
grep -E "median|identical" gpurun_out/r03h_ab_cfg5.log
