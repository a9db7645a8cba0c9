# round 3: PCPPX_WINDOW_SHORT -- its GPU parity tests, then the config 2 / 4 bench lines that use it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tuples.py tests/test_abi.py -m gpu > gpurun_out/r03j_tests.log 2>&1 || { tail -30 gpurun_out/r03j_tests.log; exit 1; }
tail -2 gpurun_out/r03j_tests.log
for c in 2 4; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline --no-e2e > gpurun_out/r03j_bench_cfg$c.json 2> gpurun_out/r03j_bench_cfg$c.err || { tail -20 gpurun_out/r03j_bench_cfg$c.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['window'], d['roofline']['frac'])" gpurun_out/r03j_bench_cfg$c.json
done
