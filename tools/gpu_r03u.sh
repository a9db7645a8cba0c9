# round 3: the whole -m gpu suite (strengthened flagged-packet parity), then file -> records and the drop-in benchmark
# after the reader changes (interleaved chains, pending starts)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03u_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03u_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03u_gpu_tests.log
timeout -k 10 1000 python -u tools/e2e_file.py --out gpurun_out/r03u_e2e_file.json > gpurun_out/r03u_e2e.log 2>&1 || { tail -20 gpurun_out/r03u_e2e.log; exit 2; }
grep -E "^map|^copy|^config1|^example|^imix" gpurun_out/r03u_e2e.log | cut -c1-420
