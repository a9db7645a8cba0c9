"""Throughput of the reassembly front ends (pcppx_reasm_device) on a parsed device batch.

  python tools/bench_reasm.py [packets] [steps]

Workload: config-3 IMIX (7/8 of the packets) followed by IP fragments / TCP segments from
tests/mutate.py:fragments (1/8) (so fragment keys and IPv6 extension replays are on the path). The parse runs
once; the timed region is `steps` reasm launches (HIP events on the launch stream). Algorithmic bytes per
packet: the 32-B summary + the packet's layer records read up to n_layers (8 B each) + 16 B written;
header bytes of fragments are counted too (<= 40 B). Also times the parse alone and the fused
parse + reassembly pass (pcppx_parse_batch_device_reasm). Prints one JSON line.
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import torch  # noqa: E402

from mutate import as_batch, fragments  # noqa: E402
from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.engine import Engine, to_device  # noqa: E402
from pcapplusplus_amd.pcap import concat  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
m = n // 8
fr = fragments(4096, 5)
b = concat([synth.config(3, n - m), as_batch([fr[i % len(fr)] for i in range(m)])])
ml = 8
eng = Engine(0)
dev = "cuda:0"
data, offsets, caplens = to_device(b, dev)
summary = torch.empty(n * 32, dtype=torch.uint8, device=dev)
layers = torch.empty(n * ml * 8, dtype=torch.uint8, device=dev)
info = torch.empty(n * 16, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev)
eng.parse_device(data, offsets, caplens, n, b.linktype, abi.make_opts(0, 8, False, ml), summary, layers, st.cuda_stream)
for _ in range(3):
    eng.reasm_device(data, offsets, caplens, n, b.linktype, summary, layers, ml, info, st.cuda_stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(steps):
    eng.reasm_device(data, offsets, caplens, n, b.linktype, summary, layers, ml, info, st.cuda_stream)
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / steps
def timed(fn):
    fn()
    torch.cuda.synchronize()
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(steps):
        fn()
    z.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(z) / steps


opts = abi.make_opts(0, 8, False, ml)
parse_ms = timed(lambda: eng.parse_device(data, offsets, caplens, n, b.linktype, opts, summary, layers, st.cuda_stream))
fused_ms = timed(lambda: eng.parse_reasm_device(data, offsets, caplens, n, b.linktype, opts, summary, layers, info,
                                                st.cuda_stream))
s = summary.view(torch.int32).view(n, 8)
nl = ((s[:, 3] >> 16) & 0xFF).clamp(max=ml).to(torch.int64)
inf = info.cpu().numpy().view(abi.REASM_DTYPE)
frag = (inf["ip_status"] & 0xF) == abi.IPR_FRAGMENT
algo = 32 * n + 8 * int(nl.sum().item()) + 16 * n + 40 * int(frag.sum())
print(json.dumps({"kernel": "reasm_kernel", "packets": n, "ms": round(ms, 4), "Gpackets_per_s": round(n / ms / 1e6, 2),
                  "algorithmic_bytes": algo, "GBps": round(algo / ms / 1e6, 1), "frac_of_8TBps": round(algo / ms / 8e9, 4),
                  "parse_only_ms": round(parse_ms, 4), "fused_parse_reasm_ms": round(fused_ms, 4),
                  "fragments": int(frag.sum()), "tcp_data": int(((inf["tcp_status"] & 0xF) == abi.TCPR_DATA).sum())}))
eng.close()
