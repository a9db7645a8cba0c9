"""Freeze the reference's 5-tuple extracts for every golden set (run in this container only).

For each tests/golden/<set>.npz, every packet parsed as Packet(&raw) by the REAL reference Packet++ (oracle/_ref,
oracle/ref_harness.cpp pcppx_ref_tuples): the first IPv4 (else IPv6) layer's addresses and protocol / nextHeader byte,
the hash5Tuple port layer's getSrcPort / getDstPort, has_5tuple and hash5Tuple (Packet++/src/PacketUtils.cpp:139-210).
Writes tests/golden/tuples/ref_tuples.npz: one structured array (include/pcppx.h pcppx_tuple) per set, keyed by the
set's file stem. Pins the restatement's extract (oracle_parse_tuples) wherever the reference library is absent.

  python tools/make_golden_tuples.py
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

OUT = ROOT / "tests" / "golden" / "tuples" / "ref_tuples.npz"


def main() -> None:
    out = {}
    for p in golden_files():
        b, _ = load_golden(p)
        out[p.stem] = oracle.ref_tuples(b)
    OUT.parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(OUT, **out)
    print(f"{OUT}: {sum(len(v) for v in out.values())} packets, {OUT.stat().st_size} B")


if __name__ == "__main__":
    main()
