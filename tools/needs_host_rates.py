"""NEEDS_HOST rate per reference capture and parse option.

The engine's flags equal the C restatement's on every packet (GPU parity tests), so the rates are computed
here on the CPU with the restatement (oracle/liboracle.so) over the reference's own captures, read by the
engine's ingest (pcppx_pcap_*). For each capture and option variant: packets, packets flagged
PCPPX_F_NEEDS_HOST (a host parse completes them), of those how many the device classified to their first
L7 layer (PCPPX_F_L7_KNOWN: HTTP / SSL / DNS for FilterTraffic's collectStats), the split by reason, and the
packets whose HTTP / SSL / DNS layers the device built itself (not flagged).

  python tools/needs_host_rates.py > profiles/r02_needs_host_rates.md
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import oracle  # noqa: E402
from pcapplusplus_amd import abi  # noqa: E402
from pcapplusplus_amd.engine import PcapReader  # noqa: E402
from pcapplusplus_amd.pcap import concat  # noqa: E402

REF = Path("/root/reference/Tests")
CAPTURES = ["Pcap++Test/PcapExamples/example.pcap", "Pcap++Test/PcapExamples/example2.pcap",
            "Pcap++Test/PcapExamples/4KHttpRequests.pcap", "Pcap++Test/PcapExamples/650HttpResponses.pcap",
            "Pcap++Test/PcapExamples/DnsPackets.pcap", "ExamplesTest/pcap_examples/tls2.pcap",
            "ExamplesTest/pcap_examples/ip-frag.pcap", "Pcap++Test/PcapExamples/sll.pcap",
            "Pcap++Test/PcapExamples/pcapng-example.pcapng"]
VARIANTS = {  # PacketParseOptions (Packet++/header/Packet.h:17-37)
    "Packet(&raw)": (0, 8),
    "Packet(&raw, TCP)": (4, 8),           # benchmark.cpp:91
    "until IP family": (0x203, 8),
    "until OSI 4": (0, 4),
    "until OSI 3": (0, 3),
}


def read(path: Path):
    out = []
    with PcapReader(path) as r:
        while True:
            b = r.read_batch(1 << 16, 64 << 20)
            if b.n == 0:
                break
            out.append(b)
    return out


def main() -> None:
    print("| capture | packets | " + " | ".join(VARIANTS) + " |")
    print("|---|---|" + "---|" * len(VARIANTS))
    for rel in CAPTURES:
        batches = read(REF / rel)
        n = sum(b.n for b in batches)
        cells = []
        for fam, osi in VARIANTS.values():
            opts = abi.make_opts(fam, osi, False, 0)
            flags, masks = [], []
            for b in batches:
                s, _ = oracle.oracle_parse(b, opts)
                flags.append(s["flags"].astype(np.uint32))
                masks.append(s["proto_mask"].astype(np.uint64))
            fl, m = np.concatenate(flags), np.concatenate(masks)
            host = (fl & abi.F_NEEDS_HOST) != 0
            l7 = host & ((fl & abi.F_NEEDS_HOST_L7) != 0)
            known = l7 & ((fl & abi.F_L7_KNOWN) != 0)
            proto = host & ((fl & abi.F_NEEDS_HOST_PROTO) != 0)
            built = (m & np.uint64((1 << 6) | (1 << 7) | (1 << 13) | (1 << 18))) != 0
            cells.append(f"{host.sum()} ({100 * host.mean():.1f}%): L7 {l7.sum()} [{known.sum()} classified], "
                         f"L2/L3 {proto.sum()}; HTTP/SSL/DNS built {built.sum()}")
        lt = sorted({b.linktype for b in batches})
        print(f"| `{rel.split('/')[-1]}` (link {','.join(map(str, lt))}) | {n} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
