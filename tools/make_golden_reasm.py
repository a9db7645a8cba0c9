"""Freeze golden vectors for the reassembly front ends (tests/golden/reasm/, run in this container only).

Expected outputs come from the REAL reference (IPReassembly::processPacket / TcpReassembly::reassemblePacket
on a first sighting, fragment keys through IPReassembly::PacketKey::getHashValue) built from /root/reference
by oracle/Makefile, through oracle/ref_harness.cpp (pcppx_ref_reasm). Inputs: the packets of the parse
golden sets (tests/golden/*.npz, reference fixture data) and a seeded fragment/TCP-segment set
(tests/mutate.py: fragments), whose bytes are stored with it.

  python tools/make_golden_reasm.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle  # noqa: E402
from conftest import golden_files, load_golden  # noqa: E402
from mutate import as_batch, fragments  # noqa: E402

OUT = ROOT / "tests" / "golden" / "reasm"


def main() -> None:
    if not oracle.ref_available():
        raise SystemExit("oracle/_ref/libpcpp_ref.so missing: `make -C oracle ref` first")
    OUT.mkdir(parents=True, exist_ok=True)
    for p in golden_files():
        if p.stem not in ("dat_ethernet", "pcap_lt1", "synth_cfg5"):
            continue
        b, _ = load_golden(p)
        np.savez_compressed(OUT / f"{p.stem}.npz", info=oracle.ref_reasm(b))
        print(p.stem, b.n)
    b = as_batch(fragments(3000, 29))
    np.savez_compressed(OUT / "fragments.npz", data=b.data, offsets=b.offsets, caplens=b.caplens,
                        linktype=np.array(b.linktype, np.int32), info=oracle.ref_reasm(b))
    print("fragments", b.n)


if __name__ == "__main__":
    main()
