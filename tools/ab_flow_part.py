"""Interleaved A/B of the partitioned flow table's count-kernel shapes (tools/ab pcppx_ab_flow_part) on config 4's
12.5M packets over their dense hash5 column; every shape's table must equal shape 0's by key.

  python tools/ab_flow_part.py [rounds]
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.engine import Engine, to_device  # noqa: E402
from tools import ab  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
b = synth.flow_stream(0, 12_500_000, 4)  # bench.py's config-4 shard (rank 0 of the one stream)
n = b.n
dev = "cuda:0"
data, offs, caps = to_device(b, dev)
st = torch.cuda.current_stream()
eng = Engine(0)
summ = torch.empty(n * 32, dtype=torch.uint8, device=dev)
fk = torch.empty(n, dtype=torch.int32, device=dev)
eng.parse_device(data, offs, caps, n, b.linktype, abi.make_opts(0, 8, False, 0, abi.WINDOW_SHORT), summ, None,
                 st.cuda_stream, fk)
cap = 1 << 21
PARTS = {6: 256, 7: 1024}  # partitions per shape (tools/ab pcppx_ab_flow_part's `want`); else 512
queues = torch.empty(1024 * (2 * ((n + 1023) // 1024) + 4096) * 4, dtype=torch.int32, device=dev)
acc = torch.zeros(cap, dtype=torch.int64, device=dev)  # shape 20's accumulator (its unpack pass leaves it zeroed)
fill = torch.zeros(512 * 256, dtype=torch.int32, device=dev)


def run(shape):
    parts = PARTS.get(shape, 512)
    rec_cap = 2 * ((n + parts - 1) // parts) + 4096
    t = (torch.zeros(cap, dtype=torch.int32, device=dev), torch.zeros(cap, dtype=torch.int64, device=dev),
         torch.zeros(cap, dtype=torch.int64, device=dev), torch.zeros(4, dtype=torch.int64, device=dev))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    abi.check(ab.lib().pcppx_ab_flow_part(abi.ptr(fk), abi.ptr(caps), n, abi.ptr(t[0]), abi.ptr(t[1]), abi.ptr(t[2]), cap,
                                          abi.ptr(t[3]), abi.ptr(acc if shape == 20 else queues), rec_cap, abi.ptr(fill),
                                          st.cuda_stream, shape),
              "pcppx_ab_flow_part")
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1), t


import os  # noqa: E402
shapes = tuple(int(x) for x in os.environ.get("AB_SHAPES", "0,5").split(","))
ref = None
for s in shapes:
    _, t = run(s)
    k = t[0].cpu().numpy().view(np.uint32)
    used = k != 0
    d = dict(zip(k[used].tolist(), zip(t[1].cpu().numpy()[used].tolist(), t[2].cpu().numpy()[used].tolist())))
    if ref is None:
        ref = d
    print(f"shape {s}: table equal to shape 0: {d == ref} ({len(d)} flows)", flush=True)
    if d != ref:
        raise SystemExit(f"shape {s}: flow table differs")
times = {s: [] for s in shapes}
for r in range(rounds):
    for s in shapes:
        ms, _ = run(s)
        if r:
            times[s].append(ms)
for s in shapes:
    t = np.array(times[s])
    print(f"shape {s}: median {np.median(t):.4f} ms  min {t.min():.4f} ms (count + merge)")
