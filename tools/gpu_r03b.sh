# round 3: new outputs (5-tuple extract, collectStats, packed layer layout) on the GPU, the whole -m gpu suite, and the
# bench lines of every config (fixed vs packed layer layout for configs 3 and 5)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tuples.py -m gpu > gpurun_out/r03b_tuples.log 2>&1 || { echo TUPLEFAIL; tail -40 gpurun_out/r03b_tuples.log; exit 1; }
tail -2 gpurun_out/r03b_tuples.log
$T 1500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests -m gpu --deselect tests/test_tuples.py > gpurun_out/r03b_gpu_tests.log 2>&1 || { echo GPUFAIL; tail -40 gpurun_out/r03b_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03b_gpu_tests.log
for a in "--config 2" "--config 4" "--config 3 --layout fixed" "--config 3 --layout packed" "--config 5 --layout fixed" "--config 5 --layout packed"; do
  tag=$(echo $a | tr -d ' -')
  $T 300 python bench.py $a --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/r03b_bench_$tag.json 2> gpurun_out/r03b_bench_$tag.err || { echo BENCHFAIL $a; tail -20 gpurun_out/r03b_bench_$tag.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print(sys.argv[2], d['value'], c['kernel_ms'], d['roofline']['frac'], d['roofline']['record_write_bytes'], c.get('collect_stats'), c.get('tuples'))" gpurun_out/r03b_bench_$tag.json "$a"
done
