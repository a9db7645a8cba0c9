"""Debug probe (GPU): the host path over batches laid out as a caller's heap would hold them -- 16-B aligned packets
with object-sized gaps, ascending or shuffled -- through pcppx_parse_batch_host (FIXED summary, DENSE + brief) against
the restatement; prints the first mismatching fields per layout.

  python tools/debug_host_layouts.py
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle  # noqa: E402
from conftest import GOLDEN, load_golden  # noqa: E402
from pcapplusplus_amd import abi  # noqa: E402
from pcapplusplus_amd.engine import Engine  # noqa: E402
from pcapplusplus_amd.pcap import PacketBatch  # noqa: E402


def heap_layout(b, shuffle: bool, seed: int = 1):
    rng = np.random.default_rng(seed)
    order = rng.permutation(b.n) if shuffle else np.arange(b.n)
    slots = [(len(b.packet(i)) + 15) // 16 * 16 + 112 for i in range(b.n)]
    pos = np.zeros(b.n, np.uint64)
    cur = 64
    for i in order:
        pos[i] = cur
        cur += slots[i]
    data = np.zeros(cur + 64, np.uint8)
    for i in range(b.n):
        p = b.packet(i)
        data[int(pos[i]):int(pos[i]) + len(p)] = np.frombuffer(p, np.uint8)
    return PacketBatch(data, pos, b.caplens.copy(), b.linktype)


def main():
    b, _ = load_golden(GOLDEN / "capture_example.npz")
    opts = abi.make_opts(0, 8, False, 16)
    os_, ol = oracle.oracle_parse(b, opts)
    with Engine(0) as eng:
        for shuffle in (False, True):
            hb = heap_layout(b, shuffle)
            for kind in ("fixed", "dense-brief", "dense-summary"):
                if kind == "fixed":
                    s, lay = eng.parse_host(hb, opts)
                    got = s
                else:
                    o = abi.make_opts(0, 8, False, 16, layout=abi.LAYOUT_DENSE)
                    s, br, dense, w = eng.parse_host_ex(hb, o, want_summary=kind == "dense-summary",
                                                        want_brief=kind == "dense-brief")
                    got = s if s is not None else br
                bad = {f: int((got[f] != os_[f]).sum()) for f in ("hash5", "hash5_dir", "hash2", "n_layers", "flags")}
                print(f"shuffle={shuffle} {kind}: mismatches {bad}", flush=True)


if __name__ == "__main__":
    main()
