"""Per-run time of the drop-in benchmark (examples/bin/benchmark) on
the reference's example.pcap at several repetition counts in one process each (GPU box, repo root): a per-run cost
that grows with the run count points at state accumulating across runs.

  python tools/dropin_reps.py [reps ...]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from pcapplusplus_amd.pcap import write_pcap  # noqa: E402


def main() -> None:
    reps = [int(a) for a in sys.argv[1:]] or [10, 110, 510, 1010]
    from conftest import GOLDEN, load_golden

    ex, _ = load_golden(GOLDEN / "capture_example.npz")
    f = Path("/dev/shm") / f"pcppx_reps_{os.getpid()}.pcap"
    write_pcap(f, ex)
    progs = {"engine": ROOT / "examples" / "bin" / "benchmark",
             "reference": ROOT / "oracle" / "_ref" / "benchmark_ref"}
    try:
        for trial in range(2):
            for name, exe in progs.items():
                if not exe.exists():
                    continue
                walls = {}
                for r in reps:
                    t = time.perf_counter()
                    subprocess.run([str(exe), str(f), "packet", str(r)], check=True, capture_output=True, timeout=600)
                    walls[r] = time.perf_counter() - t
                per = {f"{a}->{b}": round((walls[b] - walls[a]) / (b - a) * 1e3, 4) for a, b in zip(reps, reps[1:])}
                print(json.dumps({"trial": trial, "prog": name, "wall_s": {k: round(v, 3) for k, v in walls.items()},
                                  "ms_per_run": per}), flush=True)
    finally:
        f.unlink(missing_ok=True)


if __name__ == "__main__":
    main()
