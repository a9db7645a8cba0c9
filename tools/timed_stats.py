"""Kernel statistics of a bench.py run under `rocprofv3 --kernel-trace`, over the TIMED launches only.

rocprofv3's own --stats summary averages every launch of a kernel, the untimed warmup launches included. bench.py
launches the parse kernel (and, for config 4, the flow-table kernels) warmup + steps times; this tool takes the
kernel trace of the same process, keeps each such kernel's last `steps` launches (in dispatch order) and writes a
stats CSV in rocprofv3's format plus the bench line's figures beside the profile's:

  python tools/timed_stats.py <rocprof output dir> <bench stdout file>  > <tag>_kernel_stats_cfg<N>.csv

Kernels launched another number of times (one-off checks, torch helpers) are listed over all their launches; a parse
kernel launched more often than warmup + steps (the untimed check parse after the timed region runs through the same
instance) keeps launches warmup+1 .. warmup+steps.
"""
from __future__ import annotations

import csv
import json
import statistics
import sys
from pathlib import Path

HBM_PEAK_GBPS = 8000.0


def main() -> None:
    prof, bench = Path(sys.argv[1]), Path(sys.argv[2])
    traces = sorted(prof.rglob("*kernel_trace.csv"))
    if not traces:
        sys.exit(f"no kernel trace under {prof}")
    line = json.loads([ln for ln in bench.read_text().splitlines() if ln.startswith("{")][-1])
    warm, steps = int(line["warmup"]), int(line["steps"])
    launches: dict[str, list[tuple[int, int]]] = {}
    for t in traces:
        with t.open() as f:
            for r in csv.DictReader(f):
                launches.setdefault(r["Kernel_Name"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows = []
    for name, ls in launches.items():
        ls.sort()
        # the parse kernel may run once more after the timed region (bench.py's untimed check parse through the same
        # instance): launches warm+1 .. warm+steps in dispatch order are the timed ones
        timed = len(ls) == warm + steps or ("parse_tile_kernel" in name and len(ls) > warm + steps)
        use = ls[warm:warm + steps] if timed else ls
        d = [e - s for s, e in use]
        label = f"timed: last {steps} of {warm}+{steps}" if len(ls) == warm + steps else \
            f"timed: launches {warm + 1}-{warm + steps} of {len(ls)} (after them: untimed checks)"
        rows.append((name, len(d), sum(d), sum(d) / len(d), min(d), max(d), statistics.pstdev(d) if len(d) > 1 else 0.0,
                     label if timed else f"all {len(ls)}"))
    rows.sort(key=lambda r: -r[2])
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "StdDev", "Launches"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], round(r[3], 3), r[4], r[5], round(r[6], 3), r[7]])
    parse = [r for r in rows if "parse_tile_kernel" in r[0] and r[7].startswith("timed")]
    if parse:
        avg_ms = parse[0][3] / 1e6
        rb = line["roofline"]["algorithmic_read_bytes"]
        frac = rb / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
        print(f"# bench line (same process): ms_per_step {line['ms_per_step']}, kernel_ms {line['config']['kernel_ms']}, "
              f"roofline.frac {line['roofline']['frac']}; timed-launch rocprof average {avg_ms:.4f} ms -> frac "
              f"{frac:.4f} ({rb} algorithmic bytes / average / {HBM_PEAK_GBPS:.0f} GB/s); "
              f"average <= ms_per_step: {avg_ms <= line['ms_per_step']}; "
              f"profile frac within 2% of the line's: {abs(frac / line['roofline']['frac'] - 1) <= 0.02}")


if __name__ == "__main__":
    main()
