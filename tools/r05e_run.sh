set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_host_layouts.py > gpurun_out/r05e_debug.txt 2>&1; cat gpurun_out/r05e_debug.txt
AB_CASES=r04/tile-packed,tile/packed timeout -k 10 300 python -u tools/ab_kernels.py 10000000 12 3 > gpurun_out/r05e_ab_cfg3.txt 2>&1 || exit 3
tail -3 gpurun_out/r05e_ab_cfg3.txt
AB_SIZES=64 AB_CASES=r04/tile-packed,tile/packed timeout -k 10 300 python -u tools/ab_kernels.py 10000000 12 3 > gpurun_out/r05e_ab_cfg3s64.txt 2>&1 || exit 4
tail -3 gpurun_out/r05e_ab_cfg3s64.txt
AB_ML=12 AB_CASES=r04/po-packed,po/packed timeout -k 10 300 python -u tools/ab_kernels.py 10000000 12 5 > gpurun_out/r05e_ab_cfg5.txt 2>&1 || exit 5
tail -3 gpurun_out/r05e_ab_cfg5.txt
bash tools/gpu_run.sh r05e "tests:tests/test_brief.py tests/test_facade.py tests/test_gpu_parity.py::test_gpu_flow_table_partition_queue_overflow_exact" bench:3
