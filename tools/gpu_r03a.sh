set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py -k "flow" > gpurun_out/r03a_flow.log 2>&1 || { echo FLOWFAIL; tail -30 gpurun_out/r03a_flow.log; exit 1; }
tail -3 gpurun_out/r03a_flow.log
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/r03a_bench4.json 2> gpurun_out/r03a_bench4.err || { echo B4FAIL; tail -20 gpurun_out/r03a_bench4.err; exit 1; }
cat gpurun_out/r03a_bench4.json
timeout -k 10 400 python bench.py --gpus 2 --config 4 --steps 5 --warmup 2 --dist-backend gloo --no-cpu-baseline --no-e2e > gpurun_out/r03a_n2.json 2> gpurun_out/r03a_n2.err || { echo N2FAIL; tail -30 gpurun_out/r03a_n2.err; exit 1; }
cat gpurun_out/r03a_n2.json
