# round 3 final: the whole -m gpu suite on the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03final_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03final_gpu_tests.log
