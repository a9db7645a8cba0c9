# round 3: the self-launched N=2 path on one card (gloo rehearsal, both shards on the one GPU: a code-path check, not a
# scaling number) for config 3 (the driver's scaling config) and config 4 (keys-only launch + per-rank flow tables merged)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > gpurun_out/r03s_n2_cfg3.json 2> gpurun_out/r03s_n2_cfg3.err || { tail -20 gpurun_out/r03s_n2_cfg3.err; exit 1; }
tail -c 1200 gpurun_out/r03s_n2_cfg3.json
timeout -k 10 600 python -u bench.py --gpus 2 --config 4 --dist-backend gloo --steps 5 --warmup 2 > gpurun_out/r03s_n2_cfg4.json 2> gpurun_out/r03s_n2_cfg4.err || { tail -20 gpurun_out/r03s_n2_cfg4.err; exit 2; }
tail -c 1500 gpurun_out/r03s_n2_cfg4.json
