"""Phase times of the per-packet drop-in loop (GPU box, repo root): `facade_check time` on the reference's example.pcap
(frozen in tests/golden/capture_example.npz) and on BASELINE config 1's 10k pcap -- open, first getNextPacket, first
Packet(&raw, TCP) (the first page's GPU round trip), the rest of the loop, close -- to see where a small capture's run
goes next to the reference benchmark's.

  python tools/facade_probe.py [reps] [trials] [imix packets]

Each phase is the median over the trials.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from pcapplusplus_amd import synth  # noqa: E402
from pcapplusplus_amd.pcap import write_pcap  # noqa: E402


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    big = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # > 0: also config 3's IMIX pcap of that many packets
    from conftest import GOLDEN, load_golden

    progs = [(name, exe) for name, exe in (("engine", ROOT / "examples" / "bin" / "facade_check"),) if exe.exists()]
    ex, _ = load_golden(GOLDEN / "capture_example.npz")
    files = {"example.pcap": (ex, reps), "config1": (synth.config(1), reps)}
    if big:
        files["imix"] = (synth.config(3, big), 3)
    for name, (b, r) in files.items():
        f = Path("/dev/shm") / f"pcppx_probe_{os.getpid()}_{name}.pcap"
        try:
            write_pcap(f, b)
            per = {p: [] for p, _ in progs}
            for _ in range(trials):
                for pname, exe in progs:
                    res = subprocess.run([str(exe), "time", str(f), str(r)], capture_output=True, text=True, timeout=600)
                    if res.returncode != 0:
                        raise SystemExit(f"{name}: {exe.name} failed ({res.returncode}): {res.stderr[-2000:]}")
                    per[pname].append(json.loads(res.stdout.strip().splitlines()[-1]))
            for pname, ds in per.items():
                med = {k: sorted(d[k] for d in ds)[len(ds) // 2] for k in ds[0] if k.endswith("_us")}
                print(name, pname, json.dumps({"packets": ds[0]["packets"], "reps": r, "trials": trials, **med}),
                      flush=True)
        finally:
            f.unlink(missing_ok=True)


if __name__ == "__main__":
    main()
