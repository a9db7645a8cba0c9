"""Device-resident parse time of small real captures (GPU box, repo root): the reference's example.pcap (frozen in
tests/golden/capture_example.npz) and BASELINE config 1's 10k synthetic packets, under the options the drop-in
benchmark's pages use (Packet(&raw, TCP): no checksums, 16 layer records, brief + FIXED rows on the device) and with
checksums; each the median of `reps` launches timed with HIP events, plus how many packets take the generic walk (the
tools-only fast-path mark, tools/ab variant 31 / 30).

  python tools/small_capture_kernel.py [reps]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import torch  # noqa: E402

from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.engine import Engine, to_device  # noqa: E402


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    from conftest import GOLDEN, load_golden

    from tools import ab

    ex, _ = load_golden(GOLDEN / "capture_example.npz")
    out = {}
    with Engine(0) as eng:
        for name, b in (("example.pcap", ex), ("config1_10k", synth.config(1))):
            data, offs, caps = to_device(b)
            n = b.n
            summ = torch.empty(n * 32, dtype=torch.uint8, device="cuda:0")
            lay = torch.empty(n * 16 * 8, dtype=torch.uint8, device="cuda:0")
            st = torch.cuda.current_stream()
            res = {"packets": n}
            for tag, csum in (("tcp_page", False), ("checksums", True)):
                o = abi.make_opts(0, 8, csum, 16)
                ts = []
                for r in range(reps + 3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    eng.parse_device(data, offs, caps, n, b.linktype, o, summ, lay, st.cuda_stream)
                    e1.record(st)
                    torch.cuda.synchronize()
                    if r >= 3:
                        ts.append(e0.elapsed_time(e1) * 1e3)
                # packets off the fast path: the tools-only mark (flags bit 0x8000 on fast-path packets)
                ab.parse_device(data, offs, caps, n, b.linktype, o, summ, lay, st.cuda_stream, 30 if csum else 31)
                torch.cuda.synchronize()
                fl = summ.view(n, 32).view(torch.int16)[:, 6].cpu().numpy().astype(np.uint16)
                res[tag] = {"median_us": round(float(np.median(ts)), 1), "min_us": round(float(np.min(ts)), 1),
                            "generic_walk_packets": int(((fl & 0x8000) == 0).sum()),
                            "waves_with_a_generic_packet": int((((fl & 0x8000) == 0).reshape(-1)[: n // 64 * 64]
                                                                .reshape(-1, 64).any(axis=1)).sum())}
            out[name] = res
            print(name, json.dumps(res), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
