"""Per-launch table of the parse kernel's dispatches under rocprofv3 --pmc (tools/transient.py): duration, effective
shader clock = GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md, DVFS give-back: rocprofv3 sums the counter over
the 8 XCDs), and the cycle counters per dispatch.

  python tools/transient_summary.py <rocprofv3 --pmc output dir> [<plain transient.py json>]
"""
from __future__ import annotations

import csv
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path


def main() -> None:
    root = Path(sys.argv[1])
    disp: dict[int, dict] = defaultdict(dict)
    for f in sorted(root.rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "parse_tile_kernel" not in r["Kernel_Name"]:
                continue
            d = disp[int(r["Dispatch_Id"])]
            d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(disp)
    names = sorted({k for d in disp.values() for k in d if k != "ns"})
    print(f"# {len(ids)} parse dispatches under --pmc ({', '.join(names)}); clock = GRBM_GUI_ACTIVE / 8 / duration")
    print("launch  ms      clock_GHz  " + "  ".join(f"{n:>16s}" for n in names))
    rows = []
    for k, i in enumerate(ids):
        d = disp[i]
        ms = d["ns"] / 1e6
        ghz = d.get("GRBM_GUI_ACTIVE", 0.0) / 8 / d["ns"] if d["ns"] else 0.0
        rows.append((ms, ghz, d))
        print(f"{k:5d}  {ms:6.3f}  {ghz:8.3f}   " + "  ".join(f"{d.get(n, 0):16.0f}" for n in names))
    if rows:
        ms = [r[0] for r in rows]
        ghz = [r[1] for r in rows]
        print(f"# duration ms: mean {statistics.mean(ms):.4f} median {statistics.median(ms):.4f} min {min(ms):.4f} "
              f"max {max(ms):.4f}; clock GHz: min {min(ghz):.3f} max {max(ghz):.3f}")
        for n in names:
            v = [r[2].get(n, 0.0) for r in rows]
            mu = statistics.mean(v)
            print(f"# {n}: mean {mu:.0f}, min/mean {min(v) / mu:.3f}, max/mean {max(v) / mu:.3f}")
        if len(rows) > 2:
            import numpy as np

            c = np.corrcoef(np.array(ms), np.array(ghz))[0, 1]
            print(f"# correlation(duration, clock) = {c:.3f}")
    if len(sys.argv) > 2:
        plain = json.loads(Path(sys.argv[2]).read_text().strip().splitlines()[-1])
        for ph in ("phase_a", "phase_b"):
            print(f"# plain run {ph}: {plain[ph]}")


if __name__ == "__main__":
    main()
