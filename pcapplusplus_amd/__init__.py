"""pcapplusplus_amd — MI355X-native re-implementation of the Packet++ per-packet parse path.

The product path is the HIP engine (csrc/ -> libpcppx.so) behind the C ABI of include/pcppx.h;
this package holds its Python host side: the ABI mirror (abi), the engine handle (engine), pcap ingest
(pcap), the Packet++-shaped record views (packet) and synthetic workloads (synth).
"""
from . import abi
from .pcap import PacketBatch, read_pcap, write_pcap, from_packets

__all__ = ["abi", "PacketBatch", "read_pcap", "write_pcap", "from_packets"]
