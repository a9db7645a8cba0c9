"""Per-launch durations of back-to-back config-3 parse launches (the 0.80 -> 1.12 -> 0.80-ms
launch transient the headline's mean averages).

  python tools/transient.py [--launches 100] [--idle 3] [--packets 10000000] > <tag>_transient.json

Two phases in one process on the bench's own workload and launch (config 3, checksums, summary + PACKED rows, the
launch stream): `--launches` launches back to back, `--idle` seconds with the GPU idle, then `--launches` more. Each
launch is bracketed by HIP events on its stream. Run it plain (the durations) and under
`rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace` (per-dispatch cycle counters
beside the same dispatches' durations: tools/transient_summary.py) to tell clock / power management (the effective
clock GRBM_GUI_ACTIVE / 8 XCDs / duration moves with the time) from work per launch (the cycles move).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=100)
    ap.add_argument("--idle", type=float, default=3.0)
    ap.add_argument("--packets", type=int, default=10_000_000)
    args = ap.parse_args()
    import torch

    from pcapplusplus_amd import abi, synth
    from pcapplusplus_amd.engine import Engine, to_device

    dev = "cuda:0"
    batch = synth.imix(args.packets, 3)
    n = batch.n
    opts = abi.make_opts(0, 8, True, 8, abi.WINDOW_DEFAULT, abi.LAYOUT_PACKED)
    eng = Engine(0)
    data, offsets, caplens = to_device(batch, dev)
    summary = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    layers = torch.empty(n * 8 * 8, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    torch.cuda.synchronize(dev)

    def phase(k: int) -> list[float]:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        for s, e in ev:
            s.record(stream)
            eng.parse_device(data, offsets, caplens, n, batch.linktype, opts, summary, layers, sh)
            e.record(stream)
        torch.cuda.synchronize(dev)
        return [round(s.elapsed_time(e), 4) for s, e in ev]

    a = phase(args.launches)
    time.sleep(args.idle)
    b = phase(args.launches)
    eng.close()

    def stats(x):
        return {"mean": round(float(np.mean(x)), 4), "median": round(float(np.median(x)), 4),
                "min": round(float(np.min(x)), 4), "max": round(float(np.max(x)), 4),
                "first5": x[:5], "argmax": int(np.argmax(x))}

    print(json.dumps({"packets": n, "launches_per_phase": args.launches, "idle_s": args.idle,
                      "phase_a": stats(a), "phase_b": stats(b), "phase_a_ms": a, "phase_b_ms": b}), flush=True)


if __name__ == "__main__":
    main()
