"""Quick device check: runtime binding, a small bit-exact parse, and a timed full-size launch."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import oracle  # noqa: E402
from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.engine import Engine, parse_on_device, to_device  # noqa: E402

print("torch", torch.__version__, "hip", torch.version.hip, "devices", torch.cuda.device_count())
print(abi.runtime_info(0))
with open("/proc/self/maps") as f:
    print(sorted({l.split()[-1] for l in f if "amdhip64" in l or "hsa-runtime" in l}))
eng = Engine(0)
b = synth.config(3, 5000)
g = parse_on_device(eng, b)
o = oracle.oracle_parse(b)
oracle.compare_exact(g[0], g[1], o[0], o[1])
print("small parse bit-exact ok")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
b = synth.config(3, n)
data, offs, caps = to_device(b)
opts = abi.make_opts(0, 8, True, 8)
summ = torch.empty(n * 32, dtype=torch.uint8, device="cuda:0")
lay = torch.empty(n * 64, dtype=torch.uint8, device="cuda:0")
st = torch.cuda.current_stream()
for it in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    eng.parse_device(data, offs, caps, n, b.linktype, opts, summ, lay, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print(f"iter {it}: {n} pkts {ms:.3f} ms -> {n / ms / 1e3:.1f} Mpkt/s, {(int(b.caplens.sum()) + 12 * n) / ms / 1e6:.1f} GB/s")
