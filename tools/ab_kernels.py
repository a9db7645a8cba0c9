"""Interleaved A/B timing of kernel variants in one process (cdna guide §5.4 rule 24), through the tools-only
library tools/ab/libpcppx_ab.so (variant 0 = the product kernel). Records of every full variant are checked equal to
the first listed case with the same record options before timing.

  AB_CASES=po/packed,po/packed-one144 AB_ML=12 python tools/ab_kernels.py [packets] [rounds] [config]
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.engine import to_device  # noqa: E402
from tools import ab  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 10
cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 3
_sizes = __import__("os").environ.get("AB_SIZES")  # config 3 at one packet size (bench.py --sizes)
b = synth.imix(n, 3, sizes=(int(_sizes),), weights=(1,)) if _sizes else synth.config(cfg, n)
data, offs, caps = to_device(b)
summ = torch.empty(n * 32, dtype=torch.uint8, device="cuda:0")
lay = torch.empty(n * 16 * 8, dtype=torch.uint8, device="cuda:0")
st = torch.cuda.current_stream()
read_bytes = int(b.caplens.sum(dtype=np.int64)) + 12 * n  # the checksum runs' algorithmic read
_ml = int(__import__("os").environ.get("AB_ML", "8"))
PK = abi.LAYOUT_PACKED
cases = {
    # checksum instances (configs 1 / 3)
    "tile/product": (abi.make_opts(0, 8, True, 8), 0),
    "tile/packed": (abi.make_opts(0, 8, True, 8, layout=PK), 0),
    "tile/deepwin": (abi.make_opts(0, 8, True, 8, abi.WINDOW_DEEP), 0),
    "tile/deepwin-earlyB": (abi.make_opts(0, 8, True, 8, abi.WINDOW_DEEP), 70),
    "lane/ml8/csum": (abi.make_opts(0, 8, True, 8), 1),
    "tile/stream-only": (abi.make_opts(0, 8, True, 0), 2),
    "diag/tile-read": (abi.make_opts(0, 8, True, 0), 3),
    "diag/grid-read": (abi.make_opts(0, 8, True, 0), 4),
    "diag/tile-rw": (abi.make_opts(0, 8, True, 16), 7),
    # the same read + write mix under other store cache policies (round 5)
    "diag/rw-plain": (abi.make_opts(0, 8, True, 16), 120),
    "diag/rw-nt": (abi.make_opts(0, 8, True, 16), 121),
    "diag/rw-sc1": (abi.make_opts(0, 8, True, 16), 122),
    "diag/rw-sc0sc1": (abi.make_opts(0, 8, True, 16), 123),
    "diag/rw-nt-sc1": (abi.make_opts(0, 8, True, 16), 124),
    "diag/rw-nt-sc0sc1": (abi.make_opts(0, 8, True, 16), 125),
    # parse-only instances (checksums off; configs 2 / 4 / 5): records per packet AB_ML
    "po/product": (abi.make_opts(0, 8, False, _ml), 0),
    "po/packed": (abi.make_opts(0, 8, False, _ml, layout=PK), 0),
    "po/short": (abi.make_opts(0, 8, False, _ml, abi.WINDOW_SHORT), 0),
    "po/packed-short": (abi.make_opts(0, 8, False, _ml, abi.WINDOW_SHORT, PK), 0),
    "po/one144": (abi.make_opts(0, 8, False, _ml), 80),
    "po/packed-one144": (abi.make_opts(0, 8, False, _ml, layout=PK), 80),
    "po/packed-one128": (abi.make_opts(0, 8, False, _ml, layout=PK), 81),
    "po/packed-one160": (abi.make_opts(0, 8, False, _ml, layout=PK), 82),
    "po/packed-w8r6": (abi.make_opts(0, 8, False, _ml, layout=PK), 83),
    "po/gather-only": (abi.make_opts(0, 8, False, _ml), 29),
    "po/packed-gather-only": (abi.make_opts(0, 8, False, _ml, layout=PK), 29),
    # the final round-5 product kernel (tools/ab/base): round-6 changes against it in one process
    "base/tile-packed+brief": (abi.make_opts(0, 8, True, 8, layout=PK), -1),
    "base/po-packed+brief": (abi.make_opts(0, 8, False, _ml, layout=PK), -1),
    "base/po-short+tuples": (abi.make_opts(0, 8, False, 0, abi.WINDOW_SHORT), -1),
    # the 16-B brief instead of the 32-B summary (ABI 7): same rows
    "tile/packed+brief": (abi.make_opts(0, 8, True, 8, layout=PK), 0),
    "po/packed+brief": (abi.make_opts(0, 8, False, _ml, layout=PK), 0),
}
brief_t = torch.empty(n * 16, dtype=torch.uint8, device="cuda:0")
import os  # noqa: E402
only = os.environ.get("AB_CASES")
if only:
    cases = {k: v for k, v in cases.items() if k in only.split(",")}


def layer_records(o, s, l):
    """The layer records a launch defines: FIXED, the whole n x max_layers array; PACKED, each tile's run of entries
    (entries past a tile's run are not written, and a generic-walk lane's fixed-slot scratch may lie there)."""
    ml = o.max_layers
    if o.layout != PK:
        return l[: n * 8 * ml]
    nl = s.view(n, 32)[:, 14].to(torch.int64).clamp(max=ml)
    tiles = (n + 63) // 64
    cnt = torch.zeros(tiles * 64, dtype=torch.int64, device=s.device)
    cnt[:n] = nl
    tot = cnt.view(tiles, 64).sum(1)
    idx = torch.arange(n * ml, device=s.device)
    return l[: n * 8 * ml].view(torch.int64)[(idx % (64 * ml)) < tot[idx // (64 * ml)]]


# records of every full variant must equal the first listed variant's (same checksum mode), byte for byte
ref_s = ref_l = None
want_csum_ref = next(iter(cases.values()))[0].want_checksums
for name, (o, v) in cases.items():
    first = next(iter(cases.values()))[0]
    if o.max_layers != first.max_layers or o.want_checksums != want_csum_ref or o.layout != first.layout or \
            v in (2, 3, 4, 7, 29, 120, 121, 122, 123, 124, 125) or name.endswith("+brief"):  # diagnostics / other records
        continue
    summ.zero_()
    lay.zero_()
    ab.parse_device(data, offs, caps, n, b.linktype, o, summ, lay, st.cuda_stream, v)
    torch.cuda.synchronize()
    if ref_s is None:
        ref_s, ref_l = summ.clone(), layer_records(o, summ, lay).clone()
    else:
        same = torch.equal(summ, ref_s) and torch.equal(layer_records(o, summ, lay), ref_l)
        print(f"{name:18s} records identical to first variant: {same}", flush=True)
        if not same:
            raise SystemExit(f"{name}: records differ")
del ref_s, ref_l
times = {k: [] for k in cases}
for r in range(rounds):
    for name, (o, v) in cases.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        if name.endswith("+brief"):
            ab.parse_device(data, offs, caps, n, b.linktype, o, None, lay, st.cuda_stream, v, brief=brief_t)
        else:
            ab.parse_device(data, offs, caps, n, b.linktype, o, summ, lay, st.cuda_stream, v)
        e1.record(st)
        torch.cuda.synchronize()
        if r > 0:
            times[name].append(e0.elapsed_time(e1))
for name, t in times.items():
    t = np.array(t)
    # wire bytes + descriptors over the kernel time: the roofline byte model of checksum runs only (a parse-only run's
    # algorithmic read is the header extent, bench.py), so this is a rate, not a fraction of the HBM peak
    print(f"{name:18s} median {np.median(t):.4f} ms  min {t.min():.4f} ms  -> {n / np.median(t) / 1e3:8.1f} Mpkt/s"
          f"  wire+desc {read_bytes / np.median(t) / 1e6:8.1f} GB/s")
