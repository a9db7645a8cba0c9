# round 3: SkipGathered (the span stream does not re-load the chunks the header gather staged) -- records against the
# product on gapped / deep / crafted / golden batches, then the interleaved A/B on config 3
set -o pipefail
mkdir -p gpurun_out
AB_VARIANT=67 timeout -k 10 300 python -u tools/ab_check_variant.py > gpurun_out/r03v_check.log 2>&1 || { tail -20 gpurun_out/r03v_check.log; exit 1; }
tail -3 gpurun_out/r03v_check.log
AB_CASES=tile/packed,tile/packed-skipg timeout -k 10 400 python -u tools/ab_kernels.py 10000000 21 3 > gpurun_out/r03v_ab_cfg3.log 2>&1 || { tail -20 gpurun_out/r03v_ab_cfg3.log; exit 2; }
grep -E "median|identical" gpurun_out/r03v_ab_cfg3.log
AB_CASES=tile/ml8/csum,tile/fixed-skipg timeout -k 10 400 python -u tools/ab_kernels.py 10000000 11 3 > gpurun_out/r03v_ab_cfg3f.log 2>&1 || { tail -20 gpurun_out/r03v_ab_cfg3f.log; exit 3; }
grep -E "median|identical" gpurun_out/r03v_ab_cfg3f.log
