# round 3: the new bench GPU tests (configs 2 / 4 / 5 small runs through bench.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_launch.py -m gpu > gpurun_out/r03z_tests.log 2>&1 || { tail -30 gpurun_out/r03z_tests.log; exit 1; }
tail -5 gpurun_out/r03z_tests.log
