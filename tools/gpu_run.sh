#!/bin/bash
# The one GPU-box recipe (repo root on the box): each argument is a step, run in order, each under its own time limit;
# the first failing step ends the call.
#   tools/gpu_run.sh <tag> <step>...
# steps:
#   tests[:<pytest paths/-k ...>]  the -m gpu suite (default: all of tests/)  -> gpurun_out/<tag>_gpu_tests.log
#   smoke                          __graft_entry__.smoke()                      -> <tag>_smoke.log
#   e2e                            tools/e2e_file.py (file -> records, drop-in benchmark vs reference)  -> <tag>_e2e_file.json
#   bench:<cfgs>                   bench.py line per config (comma list; "3s64" etc. = config 3 at one packet size)
#   prof:<cfgs>                    the bench line under rocprofv3 --kernel-trace, plus the timed-launch-only summary
#                                  (tools/timed_stats.py) -> <tag>_prof_cfg<c>/, <tag>_kernel_stats_cfg<c>.csv
#   traffic:<cfgs>                 PMC FETCH/WRITE passes -> <tag>_traffic_cfg<c>.json (tools/measure_traffic.sh)
#   sq:<cfg>                       SQ issue counters (tools/sq_counters.sh); sqlds:<cfg> the LDS-wait / bank-conflict set
#   sqab:<cases>                   SQ issue counters of tools/ab_kernels.py cases on config 5 -> <tag>_sqab/
#   pmcab:<cases>                  one --pmc pass (PMC_COUNTERS) over tools/ab_kernels.py cases (config AB_CFG) -> <tag>_pmcab/
#   transient                      tools/transient.py plain and under rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES
#                                  SQ_BUSY_CYCLES -> <tag>_transient.json, <tag>_transient_pmc/, <tag>_transient.txt
#   ab:<cfg>:<cases>               interleaved A/B of tools/ab_kernels.py cases (comma list) on config <cfg> (3s64: config 3
#                                  at 64 B), 10M packets, 12 rounds -> <tag>_ab_cfg<cfg>.txt
#   ab6:<cfg>:<variants>           interleaved A/B of tools/ab_r06.py variants (-1 the round-5 kernel, 0 the product,
#                                  200+/210+/220+ R6 combinations) on bench.py's launch of <cfg> -> <tag>_ab6_cfg<cfg>.txt
#   cmd:<shell command>            anything else, under a 600 s limit
set -o pipefail
TAG=$1
shift
OUT=gpurun_out
ROOT=$(pwd)
mkdir -p "$OUT"
cfgargs() {  # "3s512" -> --config 3 --sizes 512
  case "$1" in
    *s*) echo "--config ${1%%s*} --sizes ${1#*s}" ;;
    *) echo "--config $1" ;;
  esac
}
SQ_DEFAULT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
tr() { [ -f "$ROOT/$OUT/${TAG}_traffic_cfg$1.json" ] && echo "--traffic $ROOT/$OUT/${TAG}_traffic_cfg$1.json"; }
for step in "$@"; do
  name=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  echo "== $step"
  case "$name" in
    tests)
      sel=${arg:-tests}
      timeout -k 10 1100 python -u -m pytest $sel -m gpu -x -v --timeout 400 --timeout-method thread \
        > "$OUT/${TAG}_gpu_tests.log" 2>&1 || { tail -40 "$OUT/${TAG}_gpu_tests.log"; exit 1; }
      tail -2 "$OUT/${TAG}_gpu_tests.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 \
        || { tail -20 "$OUT/${TAG}_smoke.log"; exit 2; }
      cat "$OUT/${TAG}_smoke.log" ;;
    e2e)
      timeout -k 10 1000 python -u tools/e2e_file.py --out "$OUT/${TAG}_e2e_file.json" $arg > "$OUT/${TAG}_e2e.log" 2>&1 \
        || { tail -20 "$OUT/${TAG}_e2e.log"; exit 3; }
      grep -E "^map|^copy|^config1|^example|^imix|^filter|^google|^first_pass" "$OUT/${TAG}_e2e.log" | cut -c1-500 ;;
    bench)
      for c in ${arg//,/ }; do
        timeout -k 10 400 python -u bench.py $(cfgargs "$c") $(tr "$c") > "$OUT/${TAG}_bench_cfg$c.json" \
          2> "$OUT/${TAG}_bench_cfg$c.err" || { tail -20 "$OUT/${TAG}_bench_cfg$c.err"; exit 4; }
        echo "cfg $c: $(head -c 400 "$OUT/${TAG}_bench_cfg$c.json")"
      done ;;
    prof)
      for c in ${arg//,/ }; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/${TAG}_prof_cfg$c" \
          -o bench --output-format csv -- python3 "$ROOT/bench.py" $(cfgargs "$c") --steps 100 --warmup 5 --no-e2e $(tr "$c") \
          > "$ROOT/$OUT/${TAG}_prof_bench_cfg$c.json" 2> "$ROOT/$OUT/${TAG}_prof_cfg$c.err") \
          || { tail -20 "$OUT/${TAG}_prof_cfg$c.err"; exit 5; }
        python3 tools/timed_stats.py "$OUT/${TAG}_prof_cfg$c" "$OUT/${TAG}_prof_bench_cfg$c.json" \
          > "$OUT/${TAG}_kernel_stats_cfg$c.csv" || exit 5
        echo "cfg $c: $(head -c 400 "$OUT/${TAG}_prof_bench_cfg$c.json")"
        cat "$OUT/${TAG}_kernel_stats_cfg$c.csv"
      done ;;
    traffic)
      for c in ${arg//,/ }; do
        tools/measure_traffic.sh "$TAG" "$c" > "$OUT/${TAG}_traffic_cfg$c.log" 2>&1 \
          || { tail -20 "$OUT/${TAG}_traffic_cfg$c.log"; exit 6; }
        grep -E '"config"|hbm_bytes|write_bytes' "$OUT/${TAG}_traffic_cfg$c.json"
      done ;;
    sq)
      tools/sq_counters.sh "$TAG" "$arg" || exit 7 ;;
    sqlds)  # LDS / memory-wait counters (the flow-table kernels)
      SQ_COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
        tools/sq_counters.sh "${TAG}lds" "$arg" || exit 7 ;;
    sqab)  # SQ issue counters of tools/ab_kernels.py cases (AB_CASES comma list) on config 5, one rocprofv3 --pmc pass
      mkdir -p "$OUT/${TAG}_sqab"
      (cd /tmp && AB_CASES="$arg" AB_ML=12 timeout -s KILL 240 rocprofv3 --pmc $SQ_DEFAULT -d "$ROOT/$OUT/${TAG}_sqab" -o p \
        --output-format csv -- python3 "$ROOT/tools/ab_kernels.py" 10000000 2 5 > "$ROOT/$OUT/${TAG}_sqab/ab.txt" \
        2> "$ROOT/$OUT/${TAG}_sqab/err.log") || { tail -20 "$OUT/${TAG}_sqab/err.log"; exit 7; }
      python3 tools/pmc_summary.py "$OUT/${TAG}_sqab" | tee "$OUT/${TAG}_sqab/summary.txt" ;;
    pmcab)  # one rocprofv3 --pmc pass (counters: PMC_COUNTERS) over tools/ab_kernels.py cases (AB_CASES=<arg>) on config AB_CFG
      mkdir -p "$OUT/${TAG}_pmcab"
      (cd /tmp && AB_CASES="$arg" timeout -s KILL 240 rocprofv3 --pmc $PMC_COUNTERS -d "$ROOT/$OUT/${TAG}_pmcab" -o p \
        --output-format csv -- python3 "$ROOT/tools/ab_kernels.py" 10000000 2 ${AB_CFG:-3} > "$ROOT/$OUT/${TAG}_pmcab/ab.txt" \
        2> "$ROOT/$OUT/${TAG}_pmcab/err.log") || { tail -20 "$OUT/${TAG}_pmcab/err.log"; exit 7; }
      python3 tools/pmc_summary.py "$OUT/${TAG}_pmcab" | tee "$OUT/${TAG}_pmcab/summary.txt" ;;
    transient)
      timeout -k 10 300 python -u tools/transient.py --launches 100 --idle 3 > "$OUT/${TAG}_transient.json" \
        2> "$OUT/${TAG}_transient.err" || { tail -20 "$OUT/${TAG}_transient.err"; exit 10; }
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        -d "$ROOT/$OUT/${TAG}_transient_pmc" -o p --output-format csv -- python3 "$ROOT/tools/transient.py" --launches 100 \
        --idle 3 > "$ROOT/$OUT/${TAG}_transient_pmc.json" 2> "$ROOT/$OUT/${TAG}_transient_pmc.err") \
        || { tail -20 "$OUT/${TAG}_transient_pmc.err"; exit 10; }
      python3 tools/transient_summary.py "$OUT/${TAG}_transient_pmc" "$OUT/${TAG}_transient.json" \
        > "$OUT/${TAG}_transient.txt" || exit 10
      tail -8 "$OUT/${TAG}_transient.txt" ;;
    ab)
      c=${arg%%:*}; cases=${arg#*:}
      case "$c" in
        *s*) sz=${c#*s}; cf=${c%%s*} ;;
        *) sz=""; cf=$c ;;
      esac
      AB_SIZES=$sz AB_ML=${AB_ML:-12} AB_CASES="$cases" timeout -k 10 400 python -u tools/ab_kernels.py 10000000 ${AB_ROUNDS:-12} "$cf" \
        > "$OUT/${TAG}_ab_cfg$c.txt" 2>&1 || { tail -20 "$OUT/${TAG}_ab_cfg$c.txt"; exit 11; }
      grep -E "median|identical" "$OUT/${TAG}_ab_cfg$c.txt" ;;
    ab6)  # round 6: interleaved A/B of tools/ab_r06.py variants on bench.py's own launch of config <cfg>
      c=${arg%%:*}; vs=${arg#*:}
      timeout -k 10 400 python -u tools/ab_r06.py "$c" "" ${AB_ROUNDS:-20} "$vs" \
        > "$OUT/${TAG}_ab6_cfg$c.txt" 2>&1 || { tail -20 "$OUT/${TAG}_ab6_cfg$c.txt"; exit 12; }
      grep -E "median|identical" "$OUT/${TAG}_ab6_cfg$c.txt" ;;
    cmd)
      timeout -k 10 600 bash -c "$arg" || exit 8 ;;
    *)
      echo "unknown step $step"; exit 9 ;;
  esac
done
echo "gpu_run $TAG ok"
