"""Interleaved A/B of parse-only instances on BASELINE config 2 (1M x 64 B) writing the 5-tuple extract alone, as
bench.py --config 2 does (tools/ab/libpcppx_ab.so; variant 0 = the product's launch).

  AB_VARIANTS=0,60,61 python tools/ab_cfg2.py [packets] [rounds]
"""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.engine import to_device  # noqa: E402
from tools import ab  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 50
cfg = int(os.environ.get("AB_CONFIG", "2"))
variants = [int(v) for v in os.environ.get("AB_VARIANTS", "0,60,61,62,63,64").split(",")]
b = synth.config(cfg, n)
data, offs, caps = to_device(b)
tup = torch.empty(n * 48, dtype=torch.uint8, device="cuda:0")
st = torch.cuda.current_stream()
o = abi.make_opts(0, 8, False, 0)
ref = None
for v in variants:
    tup.fill_(0xAB)
    ab.parse_device(data, offs, caps, n, b.linktype, o, None, None, st.cuda_stream, v, tuples=tup)
    torch.cuda.synchronize()
    if ref is None:
        ref = tup.clone()
    elif not torch.equal(tup, ref):
        raise SystemExit(f"variant {v}: tuples differ from variant {variants[0]}")
print(f"tuples identical across variants {variants}", flush=True)
times = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        ab.parse_device(data, offs, caps, n, b.linktype, o, None, None, st.cuda_stream, v, tuples=tup)
        e1.record(st)
        torch.cuda.synchronize()
        if r > 0:
            times[v].append(e0.elapsed_time(e1))
for v, t in times.items():
    t = np.array(t)
    print(f"variant {v:3d} median {np.median(t) * 1e3:8.2f} us  min {t.min() * 1e3:8.2f} us  -> "
          f"{n / np.median(t) / 1e3:8.1f} Mpkt/s", flush=True)
