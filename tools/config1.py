"""BASELINE config 1 (plumbing): a 10k-packet Eth/IPv4/UDP pcap through the reference's own
Examples/PcapPlusPlus-benchmark (oracle/_ref/benchmark_ref, compiled unchanged by `make -C oracle bench`) and
through the engine's drop-in of the same program (examples/bin/benchmark: batch prepass on the GPU, needs one).

The reference prints "<packets per run> <integer ms per run>"; 10k packets take ~1 ms, so each program is run
with R1 and R2 repetitions and the per-run time is the wall-clock difference / (R2 - R1) (process start-up,
file open and, for the engine, HIP initialisation cancel out).

  python tools/config1.py [--gpu] [--out profiles/r02_config1.json]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from pcapplusplus_amd import synth  # noqa: E402
from pcapplusplus_amd.pcap import write_pcap  # noqa: E402


def per_run_ms(exe: Path, pcap: Path, r1: int, r2: int, extra=()) -> tuple[float, str]:
    def wall(reps: int) -> tuple[float, str]:
        t = time.perf_counter()
        out = subprocess.run([str(exe), str(pcap), "packet", str(reps), *extra], capture_output=True, text=True,
                             check=True, timeout=600).stdout.strip().splitlines()[-1]
        return time.perf_counter() - t, out
    w1, _ = wall(r1)
    w2, out = wall(r2)
    return (w2 - w1) / (r2 - r1) * 1e3, out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", action="store_true", help="also run examples/bin/benchmark (needs a GPU)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    b = synth.config(1)
    pcap = Path(tempfile.mkdtemp()) / "config1.pcap"
    write_pcap(pcap, b)
    res = {"config": "BASELINE config 1: 10k-packet pcap, Eth/IPv4/UDP, Examples/PcapPlusPlus-benchmark packet mode "
                     "(Packet(&raw, TCP) per packet)", "packets": b.n, "pcap_bytes": pcap.stat().st_size}
    ref = ROOT / "oracle" / "_ref" / "benchmark_ref"
    if ref.exists():
        ms, out = per_run_ms(ref, pcap, 10, 2010)
        res["reference_benchmark"] = {"ms_per_run": round(ms, 4), "Mpackets_per_s": round(b.n / ms / 1e3, 2),
                                      "stdout": out, "threads": 1,
                                      "what": "reference benchmark.cpp unchanged: PcapFileReaderDevice::getNextPacket + "
                                              "Packet(&raw, TCP), one core"}
    if args.gpu:
        ex = ROOT / "examples" / "bin" / "benchmark"
        ms, out = per_run_ms(ex, pcap, 10, 510)
        res["engine_benchmark"] = {"ms_per_run": round(ms, 4), "Mpackets_per_s": round(b.n / ms / 1e3, 2),
                                   "stdout": out,
                                   "what": "examples/benchmark.cpp: pcap batch read + pcppx_parse_batch_host (H2D, "
                                           "parse, D2H) + the per-packet handler, per run"}
    line = json.dumps(res, indent=1)
    print(line)
    if args.out:
        Path(args.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
