# round 3 final: the driver's own commands on the final tree -- smoke(), then plain `python bench.py`
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03w_smoke.log 2>&1 || { tail -20 gpurun_out/r03w_smoke.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03w_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r03w_bench.json 2> gpurun_out/r03w_bench.err || { tail -20 gpurun_out/r03w_bench.err; exit 2; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['traffic'], r['traffic_source'][:40], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])" gpurun_out/r03w_bench.json
