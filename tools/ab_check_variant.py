"""TOOLS ONLY: a parse variant of tools/ab/libpcppx_ab.so against the product launch on batches beyond the A/B's packed
config-3 batch -- gapped (every start alignment, HBM edge chunks), deep stacks with checksums, crafted and L7 stacks,
config-3 batches with gaps of zero bytes, every golden set -- records equal byte for byte (summary and layers).

  AB_VARIANT=<n> python tools/ab_check_variant.py   (variant 67, SkipGathered, lives in commit history: profiles/r03_ab_skip_gathered.txt)
"""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
import torch  # noqa: E402

from conftest import golden_files, load_golden  # noqa: E402
from mutate import as_batch, crafted, crafted_l7  # noqa: E402
from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.engine import to_device  # noqa: E402
from tools import ab  # noqa: E402

V = int(os.environ.get("AB_VARIANT", "67"))


def run(batch, opts, variant):
    data, offs, caps = to_device(batch)
    n = batch.n
    s = torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device="cuda:0")
    lay = torch.zeros(max(n * opts.max_layers, 1) * 8, dtype=torch.uint8, device="cuda:0")
    ab.parse_device(data, offs, caps, n, batch.linktype, opts, s, lay, torch.cuda.current_stream().cuda_stream, variant)
    torch.cuda.synchronize()
    return s.cpu().numpy(), lay.cpu().numpy()


def same(batch, opts, what):
    a = run(batch, opts, 0)
    b = run(batch, opts, V)
    ok = np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    print(f"{what:40s} n={batch.n:8d} equal={ok}", flush=True)
    if not ok:
        raise SystemExit(f"variant {V} differs on {what}")


for layout in (abi.LAYOUT_FIXED, abi.LAYOUT_PACKED):
    o = abi.make_opts(0, 8, True, 8, layout=layout)
    b3 = synth.config(3, 300_000)
    same(b3, o, f"config 3 packed batch, layout {layout}")
    g = as_batch([b3.packet(i) for i in range(60_000)], gaps=True, seed=3)
    same(g, o, f"config 3 gapped, layout {layout}")
    b5 = synth.config(5, 100_000)
    same(b5, abi.make_opts(0, 8, True, 12, layout=layout), f"config 5 with checksums, layout {layout}")
    c = as_batch(crafted() + crafted_l7(), gaps=False, seed=7)
    same(c, abi.make_opts(0, 8, True, 16 if layout == abi.LAYOUT_FIXED else 12, layout=layout), f"crafted, layout {layout}")
    cg = as_batch(crafted() + crafted_l7(), gaps=True, seed=8)
    same(cg, abi.make_opts(0, 8, True, 16 if layout == abi.LAYOUT_FIXED else 12, layout=layout), f"crafted gapped, layout {layout}")
for path in golden_files():
    batch, variants = load_golden(path)
    for v, (opts, rsum, rlay) in variants.items():
        if opts.want_checksums:
            same(batch, opts, f"{path.stem}/{v}")
print("all equal")
