# round 3: config 4's summary-free flow launch (dense keys + collectStats) -- GPU test, traffic, bench line + rocprof
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tuples.py -m gpu -k "summary_free or short_window" > gpurun_out/r03o_tests.log 2>&1 || { tail -30 gpurun_out/r03o_tests.log; exit 1; }
tail -2 gpurun_out/r03o_tests.log
tools/measure_traffic.sh r03o 4 > gpurun_out/r03o_traffic.log 2>&1 || { tail -20 gpurun_out/r03o_traffic.log; exit 2; }
cp gpurun_out/r03o_traffic_cfg4.json profiles/traffic_cfg4.json
tools/bench_all.sh r03o 4 > gpurun_out/r03o_bench_all.log 2>&1 || { tail -20 gpurun_out/r03o_bench_all.log; exit 3; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], c['records'], c['window'], d['roofline']['frac'], d['roofline']['traffic'], c.get('flow_keys_equal_hash5'), c['flow_table']['exact'], c['collect_stats']['consistent'])" gpurun_out/r03o_bench_cfg4.json
AB_CASES=tile/packed,diag/tile-read,diag/tile-rw timeout -k 10 400 python -u tools/ab_kernels.py 10000000 15 3 > gpurun_out/r03o_ab_floor.log 2>&1 || { tail -20 gpurun_out/r03o_ab_floor.log; exit 4; }
grep -E "median" gpurun_out/r03o_ab_floor.log
AB_SHAPES=0,5,8 timeout -k 10 400 python -u tools/ab_flow_part.py 15 > gpurun_out/r03o_ab_flow.log 2>&1 || { tail -20 gpurun_out/r03o_ab_flow.log; exit 5; }
grep -v amdgpu.ids gpurun_out/r03o_ab_flow.log
