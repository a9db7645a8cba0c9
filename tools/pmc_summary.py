"""Summarise rocprofv3 --pmc CSVs: per kernel-dispatch counter values (averaged over dispatches of the
same kernel+grid), with derived per-wave numbers."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
rows = defaultdict(lambda: defaultdict(list))
order = []
for f in sorted(root.rglob("*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        name = next((x for x in ("parse_tile_kernel", "parse_lane_kernel", "diag_tile_read", "diag_grid_read",
                                 "flow_count_kernel") if x in kn), kn[:40])
        key = (name, int(r["Dispatch_Id"]) if False else 0, r["Grid_Size"])
        disp = (f.parent.name, r["Dispatch_Id"])
        rows[(name, r["Grid_Size"])][r["Counter_Name"]].append((disp, float(r["Counter_Value"]),
                                                                int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
for (name, grid), ctr in rows.items():
    print(f"== {name} grid={grid}")
    for c, vals in sorted(ctr.items()):
        v = [x[1] for x in vals]
        print(f"  {c:24s} n={len(v):3d} mean={sum(v) / len(v):16.1f}")
