# round 3: the capture-file -> records example and the end-to-end rates (tools/e2e_file.py)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_examples.py -m gpu > gpurun_out/r03c_examples.log 2>&1 || { echo EXFAIL; tail -40 gpurun_out/r03c_examples.log; exit 1; }
tail -2 gpurun_out/r03c_examples.log
$T 1000 python -u tools/e2e_file.py --out gpurun_out/r03c_e2e_file.json > gpurun_out/r03c_e2e.log 2>&1 || { echo E2EFAIL; tail -40 gpurun_out/r03c_e2e.log; exit 1; }
tail -60 gpurun_out/r03c_e2e.log
