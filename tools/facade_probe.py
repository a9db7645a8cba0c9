"""Phase times of the per-packet drop-in loop (GPU box, repo root): `facade_check time` on the reference's example.pcap
(frozen in tests/golden/capture_example.npz) and on BASELINE config 1's 10k pcap -- open, first getNextPacket, first
Packet(&raw, TCP) (the first page's GPU round trip), the rest of the loop, close -- to see where a small capture's run
goes next to the reference benchmark's.

  python tools/facade_probe.py [reps]
"""
from __future__ import annotations

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
    from conftest import GOLDEN, load_golden

    ex, _ = load_golden(GOLDEN / "capture_example.npz")
    files = {"example.pcap": ex, "config1": synth.config(1)}
    for name, b in files.items():
        f = Path("/dev/shm") / f"pcppx_probe_{os.getpid()}_{name}.pcap"
        try:
            write_pcap(f, b)
            r = subprocess.run([str(ROOT / "examples" / "bin" / "facade_check"), "time", str(f), str(reps)],
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise SystemExit(f"{name}: facade_check failed ({r.returncode}): {r.stderr[-2000:]}")
            print(name, r.stdout.strip(), flush=True)
        finally:
            f.unlink(missing_ok=True)


if __name__ == "__main__":
    main()
