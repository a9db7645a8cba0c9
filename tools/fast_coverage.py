"""TOOLS ONLY: which packets of a synthetic config the fast path takes (tools/ab variants 30/31 mark them), broken
down by layer stack.

  python tools/fast_coverage.py <config> [packets]
"""
import sys
from collections import Counter
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from pcapplusplus_amd import abi, synth  # noqa: E402
from tools import ab  # noqa: E402

cfg = int(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
b = synth.config(cfg, n)
for variant, csum in ((30, True), (31, False)):
    s, lay = ab.parse_on_device(b, abi.make_opts(0, 8, csum, 12), variant)
    fast = (s["flags"] & 0x8000) != 0
    stacks = Counter()
    slow = Counter()
    for i in range(b.n):
        key = "/".join(str(int(x)) for x in lay[i][: min(int(s["n_layers"][i]), 12)]["proto"])
        stacks[key] += 1
        if not fast[i]:
            slow[key] += 1
    print(f"variant {variant} (checksums {csum}): fast {fast.mean():.4f} of {b.n}")
    for k, v in slow.most_common(12):
        print(f"   slow {v:7d} of {stacks[k]:7d}  {k}")
    mis = (b.offsets & 15)[~fast]
    print("   slow packets by start offset mod 16:", np.bincount(mis.astype(np.int64), minlength=16).tolist())
