"""The C++ example programs over pcppx.hpp (examples/): the reference's benchmark packet mode and the
FilterTraffic worker over a pcap file. GPU runs compare with the reference worker / the restatement."""
from __future__ import annotations

import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from conftest import ROOT
from pcapplusplus_amd import abi, synth
from pcapplusplus_amd.pcap import read_pcap, write_pcap

BIN = ROOT / "examples" / "bin"


def run(args, timeout=300):
    return subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=timeout)


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-C", str(ROOT / "examples")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return BIN


def test_usage_without_device(built):
    r = run([built / "benchmark"])
    assert r.returncode == 1 and "Usage" in r.stdout
    r = run([built / "filter_traffic", "-f"])
    assert r.returncode == 1 and "Usage" in r.stdout
    r = run([built / "filter_traffic", "-f", "x.pcap", "-P", "ICMP"])
    assert r.returncode == 1


def stats_from(text: str) -> dict:
    names = {"Eth count": "eth_count", "ARP count": "arp_count", "IPv4 count": "ipv4_count",
             "IPv6 count": "ipv6_count", "TCP count": "tcp_count", "UDP count": "udp_count",
             "Matched TCP flows": "matched_tcp_flows", "Matched UDP flows": "matched_udp_flows",
             "Total packet count": "packet_count", "Matched packet count": "matched_packets"}
    out = {}
    for m in re.finditer(r"\|\s*([A-Za-z0-9 ]+?)\s*\|\s*(\d+)\s*\|", text):
        if m.group(1) in names:
            out[names[m.group(1)]] = int(m.group(2))
    return out


@pytest.mark.gpu
def test_benchmark_packet_mode(built, tmp_path):
    b = synth.config(3, 300_000)
    f = tmp_path / "in.pcap"
    write_pcap(f, b)
    r = run([built / "benchmark", f, "packet", 3])
    assert r.returncode == 0, r.stderr
    count, ms = (int(x) for x in r.stdout.split())
    assert count == b.n


@pytest.mark.gpu
def test_filter_traffic_tool(built, tmp_path):
    b = synth.imix(50_000, 23, flows=2000, corrupt_frac=0.0)
    f, o = tmp_path / "in.pcap", tmp_path / "out.pcap"
    write_pcap(f, b)
    # a destination port seen in the data, TCP only
    s, lay = oracle.oracle_parse(b.slice(0, 1000), abi.make_opts(0, 8, False, 16))
    k = int(np.nonzero(s["proto_mask"] & (1 << 4))[0][0])
    l4 = [int(x["offset"]) for x in lay[k] if x["proto"] == 4][0]
    pkt = b.packet(k)
    dport = pkt[l4 + 2] << 8 | pkt[l4 + 3]
    r = run([built / "filter_traffic", "-f", f, "-o", o, "-D", dport, "-P", "TCP"])
    assert r.returncode == 0, r.stderr
    spec = oracle.make_spec(dst_port=dport, protocol=4)
    if oracle.ref_available():
        want_m, want = oracle.ref_filter(b, spec)
    else:
        s, lay = oracle.oracle_parse(b, abi.make_opts(0, 8, False, 16), threads=8)
        want_m, want = oracle.oracle_filter(b, s, lay, spec)
    got = stats_from(r.stdout)
    for key, v in got.items():
        assert v == want[key], (key, v, want[key])
    w = read_pcap(o)
    assert [w.packet(i) for i in range(w.n)] == [b.packet(i) for i in np.nonzero(want_m)[0]]
