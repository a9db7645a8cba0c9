"""Summarise rocprofv3 --pmc CSVs: per kernel instance (template arguments kept, so the parse kernel's instances are
not mixed: a parse-only bench run also launches the checksum instance once for its header-extent model) and grid,
the counter values averaged over that instance's dispatches, with per-wave figures.

  python tools/pmc_summary.py <rocprofv3 output dir>
"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def short(kn: str) -> str:
    for x in ("parse_tile_kernel", "parse_lane_kernel", "diag_tile_read", "diag_grid_read", "flow_count_kernel",
              "flow_merge_kernel", "proto_stats_reduce_kernel"):
        if x in kn:
            kn = re.sub(r"pcppx::\(anonymous namespace\)::", "", kn)
            m = re.search(re.escape(x) + r"<([^()]*)>", kn)
            args = m.group(1) if m else ""
            return f"{x}<{args}>" if args else x
    return kn[:40]


root = Path(sys.argv[1])
rows = defaultdict(lambda: defaultdict(list))
for f in sorted(root.rglob("*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        rows[(short(r["Kernel_Name"]), r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (name, grid), ctr in rows.items():
    waves = (int(grid) + 63) // 64
    print(f"== {name} grid={grid} ({waves} waves)")
    for c, v in sorted(ctr.items()):
        mean = sum(v) / len(v)
        print(f"  {c:24s} n={len(v):3d} mean={mean:16.1f}  per wave={mean / waves:10.1f}")
