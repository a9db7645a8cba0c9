# round 3: file -> records and the drop-in benchmark after the reader changes (interleaved chains, pending starts)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/e2e_file.py --out gpurun_out/r03t_e2e_file.json > gpurun_out/r03t_e2e.log 2>&1 || { tail -20 gpurun_out/r03t_e2e.log; exit 1; }
grep -E "^map|^copy|^config1|^example|^imix" gpurun_out/r03t_e2e.log | cut -c1-400
