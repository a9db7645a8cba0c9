"""Collect the reference's own packet fixtures (data files only) into packed batches.

Used in this container only (it reads /root/reference) by tools/make_golden.py, which freezes the
inputs together with the reference's outputs under tests/golden/.
"""
from __future__ import annotations

from pathlib import Path

from pcapplusplus_amd import abi
from pcapplusplus_amd.pcap import PacketBatch, from_packets, read_hex_dat, read_pcap

REF = Path("/root/reference")
DAT_DIR = REF / "Tests/Packet++Test/PacketExamples"
PCAP_DIRS = [REF / "Tests/Packet++Test/PacketExamples", REF / "Tests/Pcap++Test/PcapExamples",
             REF / "Tests/ExamplesTest/pcap_examples"]
FUZZ_DIR = REF / "Tests/Fuzzers/RegressionTests/regression_samples"


def dat_batch() -> PacketBatch:
    files = sorted(DAT_DIR.glob("*.dat"))
    pk, names = [], []
    for f in files:
        try:
            pk.append(read_hex_dat(f))
            names.append(f.name)
        except ValueError:
            continue
    b = from_packets(pk, abi.LINKTYPE_ETHERNET)
    b.meta["names"] = names
    return b


def pcap_batches(max_packets: int | None = None) -> dict[str, PacketBatch]:
    out = {}
    for d in PCAP_DIRS:
        if not d.exists():
            continue
        for f in sorted(list(d.glob("*.pcap")) + list(d.glob("*.cap"))):
            try:
                b = read_pcap(f, max_packets)
            except (ValueError, OSError):
                continue
            if b.n:
                out[f"{d.parent.name}/{f.name}"] = b
    return out


def fuzz_batches() -> dict[str, PacketBatch]:
    out = {}
    for f in sorted(FUZZ_DIR.glob("*")) if FUZZ_DIR.exists() else []:
        try:
            b = read_pcap(f)
        except (ValueError, OSError, Exception):
            continue
        if b.n:
            out[f"fuzz/{f.name}"] = b
    return out
