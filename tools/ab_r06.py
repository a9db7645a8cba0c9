"""Interleaved A/B of parse kernels on bench.py's own launches (records as bench.py writes them), in one process
(cdna guide §5.4 rule 24): the final round-5 kernel (tools/ab/base, variant -1) against today's product kernel
(variant 0 of tools/ab/libpcppx_ab.so, which compiles the product source) and any tools-only variants. Every case's
records are checked equal, byte for byte, to the first case's before timing.

  python tools/ab_r06.py <config> [packets] [rounds] [variants]      config: 2 | 3 | 3s64 | 3s512 | 3s1500 | 4 | 5
  (variant -2: the round-6 kernel before the Cisco HDLC / NFLOG first layers, tools/ab/base/libpcppx_base6.so)
  e.g. python tools/ab_r06.py 3s64 10000000 20 -1,0
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.engine import to_device  # noqa: E402
from tools import ab  # noqa: E402

cfg_arg = sys.argv[1] if len(sys.argv) > 1 else "3"
cfg = int(cfg_arg[0])
sized = int(cfg_arg[2:]) if "s" in cfg_arg else None
n = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] else {2: 1_000_000, 3: 10_000_000, 4: 12_500_000, 5: 10_000_000}[cfg]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 20
variants = [int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "-1,0").split(",")]

if cfg == 3:
    b = synth.imix(n, 3, sizes=(sized,), weights=(1,)) if sized else synth.imix(n, 3)
elif cfg == 4:
    b = synth.flow_stream(0, n, 4)
elif cfg == 5:
    b = synth.deep(n, 5)
else:
    b = synth.small64(n, 2)
PK = abi.LAYOUT_PACKED
# bench.py's launch per config (CONFIG_MAX_LAYERS / CONFIG_LAYOUT / CONFIG_RECORDS / CONFIG_WINDOW)
if cfg == 3:
    opts, kind = abi.make_opts(0, 8, True, 8, abi.WINDOW_DEFAULT, PK), "brief"
elif cfg == 5:
    opts, kind = abi.make_opts(0, 8, False, 12, abi.WINDOW_DEFAULT, PK), "brief"
elif cfg == 4:
    opts, kind = abi.make_opts(0, 8, False, 0, abi.WINDOW_SHORT), "keys"
else:
    opts, kind = abi.make_opts(0, 8, False, 0, abi.WINDOW_SHORT), "tuples"
data, offs, caps = to_device(b)
st = torch.cuda.current_stream()
ml = opts.max_layers
lay = torch.empty(max(n * max(ml, 1), 1) * 8, dtype=torch.uint8, device="cuda:0")
brief = torch.empty(n * 16, dtype=torch.uint8, device="cuda:0") if kind == "brief" else None
tup = torch.empty(n * 48, dtype=torch.uint8, device="cuda:0") if kind == "tuples" else None
keys = torch.empty(n, dtype=torch.int32, device="cuda:0") if kind == "keys" else None


def launch(v):
    ab.parse_device(data, offs, caps, n, b.linktype, opts, None, lay if ml else None, st.cuda_stream, v,
                    tuples=tup, brief=brief, flow_keys=keys)


def records():
    if kind == "tuples":
        return [tup.clone()]
    if kind == "keys":
        return [keys.clone()]
    nl = brief.view(n, 16)[:, 14].to(torch.int64).clamp(max=ml)  # n_layers byte of the brief
    tiles = (n + 63) // 64
    cnt = torch.zeros(tiles * 64, dtype=torch.int64, device="cuda:0")
    cnt[:n] = nl
    tot = cnt.view(tiles, 64).sum(1)
    idx = torch.arange(n * ml, device="cuda:0")
    rows = lay[: n * 8 * ml].view(torch.int64)[(idx % (64 * ml)) < tot[idx // (64 * ml)]]
    return [brief.clone(), rows.clone()]


DIAG = {270, 271}  # diagnostics whose records differ by design (half of each PACKED run stored)
ref = None
for v in variants:
    lay.fill_(0xAB)
    for t in (brief, tup, keys):
        if t is not None:
            t.fill_(0x5A)
    launch(v)
    torch.cuda.synchronize()
    got = records()
    if v in DIAG:
        print(f"variant {v}: diagnostic, records not compared", flush=True)
    elif ref is None:
        ref = got
    else:
        same = all(torch.equal(a, c) for a, c in zip(got, ref))
        print(f"variant {v}: records identical to variant {variants[0]}: {same}", flush=True)
        if not same:
            raise SystemExit(f"variant {v}: records differ")
del ref
# short kernels (config 2: ~30 us) are timed as `reps` back-to-back launches per sample, so that launch gaps and the
# clock's response to one short burst do not decide the comparison
reps = max(1, int(2_000_000 // n))
times = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            launch(v)
        e1.record(st)
        torch.cuda.synchronize()
        if r > 0:
            times[v].append(e0.elapsed_time(e1) / reps)
print(f"config {cfg_arg}: {n} packets, {rounds - 1} interleaved rounds of {reps} launches, records {kind}", flush=True)
for v, t in times.items():
    t = np.array(t)
    print(f"variant {v:4d} median {np.median(t):.4f} ms  min {t.min():.4f} ms  mean {t.mean():.4f} ms  -> "
          f"{n / np.median(t) / 1e3:8.1f} Mpkt/s", flush=True)
