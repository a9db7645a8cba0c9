"""Freeze golden parity fixtures under tests/golden/ (run in this container only).

Inputs are data files the reference's own tests hold (Tests/Packet++Test/PacketExamples/*.dat|*.pcap,
Tests/Pcap++Test/PcapExamples/*.pcap, Tests/Fuzzers/RegressionTests/regression_samples) plus small
seed-generated synthetic batches. Expected outputs come from the REAL reference Packet++ (built from
/root/reference sources by oracle/Makefile into oracle/_ref/libpcpp_ref.so) through oracle/ref_harness.cpp.

  python tools/make_golden.py            # everything
  python tools/make_golden.py captures   # only the whole-capture fixtures (CAPTURES)

Writes tests/golden/<name>.npz with: data, offsets, caplens, linktype, set_names, set_index,
and per option variant v: sum_<v>, lay_<v> (reference records), opts_<v> (family, osi, csum, max_layers).
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import oracle  # noqa: E402
from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.pcap import PacketBatch, from_packets  # noqa: E402
from tools import corpus  # noqa: E402

OUT = Path(__file__).resolve().parents[1] / "tests" / "golden"

# parse-option variants pinned by the golden records (PacketParseOptions, Packet++/header/Packet.h:17-37)
VARIANTS = {
    "full": (0, 8, 1, 16),
    "until_tcp": (4, 8, 1, 16),          # Packet(&raw, TCP) as benchmark.cpp:91-94
    "until_ip": (0x203, 8, 1, 16),       # ProtocolTypeFamily IP
    "until_osi3": (0, 3, 1, 16),         # OsiModelNetworkLayer
    "until_osi2": (0, 2, 0, 8),
    "no_layers": (0, 8, 1, 0),
}
PER_PCAP_LIMIT = 250


def merge(named: dict[str, PacketBatch]) -> tuple[PacketBatch, list[str], np.ndarray]:
    names, pk, idx = [], [], []
    for k, (name, b) in enumerate(named.items()):
        names.append(name)
        for i in range(b.n):
            pk.append(b.packet(i))
            idx.append(k)
    lt = next(iter(named.values())).linktype
    return from_packets(pk, lt), names, np.array(idx, dtype=np.int32)


def dump(name: str, batch: PacketBatch, set_names: list[str], set_index: np.ndarray, variants=VARIANTS) -> None:
    out = {"data": batch.data, "offsets": batch.offsets, "caplens": batch.caplens,
           "linktype": np.array(batch.linktype, np.int32), "set_names": np.array(set_names),
           "set_index": set_index}
    for v, (fam, osi, cs, ml) in variants.items():
        opts = abi.make_opts(fam, osi, bool(cs), ml)
        s, lay = oracle.ref_parse(batch, opts)
        out[f"sum_{v}"] = s
        out[f"lay_{v}"] = lay
        out[f"opts_{v}"] = np.array([fam, osi, cs, ml], np.int64)
    OUT.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(OUT / f"{name}.npz", **out)
    print(f"{name}: {batch.n} packets, {batch.data.nbytes} bytes -> {(OUT / f'{name}.npz').stat().st_size} B")


# whole captures of the reference's Pcap++ tests, each in its own fixture (the example programs' parity tests)
CAPTURES = {"capture_example": "Tests/Pcap++Test/PcapExamples/example.pcap"}


def dump_captures() -> None:
    from pcapplusplus_amd.pcap import read_pcap

    for name, rel in CAPTURES.items():
        b = read_pcap(corpus.REF / rel)
        dump(name, b, [rel], np.zeros(b.n, np.int32))


def main() -> None:
    if not oracle.ref_available():
        raise SystemExit("oracle/_ref/libpcpp_ref.so missing: `make -C oracle ref` first")
    if sys.argv[1:] == ["captures"]:
        dump_captures()
        return
    dump_captures()
    # 1. single-packet .dat fixtures (Ethernet)
    d = corpus.dat_batch()
    dump("dat_ethernet", d, d.meta["names"], np.arange(d.n, dtype=np.int32))
    # 2. pcap fixtures grouped by link type (example2.pcap whole; others capped)
    by_lt: dict[int, dict[str, PacketBatch]] = {}
    for name, b in corpus.pcap_batches().items():
        if not name.endswith("example2.pcap") and b.n > PER_PCAP_LIMIT:
            b = b.slice(0, PER_PCAP_LIMIT)
        by_lt.setdefault(b.linktype, {})[name] = b
    for name, b in corpus.fuzz_batches().items():
        by_lt.setdefault(b.linktype, {})[name] = b
    for lt, named in sorted(by_lt.items()):
        batch, names, idx = merge(named)
        dump(f"pcap_lt{lt}", batch, names, idx)
    # 3. small synthetic batches of every config shape
    for cfg, n in ((1, 400), (2, 3000), (3, 1500), (4, 1000), (5, 1000)):
        b = synth.config(cfg, n)
        dump(f"synth_cfg{cfg}", b, [f"config{cfg}"], np.zeros(b.n, np.int32), {"full": VARIANTS["full"]})


if __name__ == "__main__":
    main()
