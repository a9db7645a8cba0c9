# round 3: stream-first A/B of the checksum instance (config 3, packed layout), records checked identical
set -o pipefail
mkdir -p gpurun_out
AB_CASES=tile/packed,tile/packed-sf,tile/packed-sf-cached,tile/packed-sf-w6 timeout -k 10 500 python -u tools/ab_kernels.py 10000000 15 3 > gpurun_out/r03e_ab_sf.log 2>&1 || { tail -20 gpurun_out/r03e_ab_sf.log; exit 2; }
grep -E "median|identical" gpurun_out/r03e_ab_sf.log
