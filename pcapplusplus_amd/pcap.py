"""pcap ingest/egest into packed packet batches.

Follows the reference's file rules (Pcap++/src/PcapFileDevice.cpp): magic detection and byte swapping
(:53-60, :667-705), 16-byte record headers (:66-87), and the record checks of readNextPacket
(:799-880): caplen > len, caplen > 256 KiB, or a sub-second field out of range end the read; caplen
beyond the snapshot length is truncated. Packets land back to back in one byte array, which is the
layout the device kernels stream best.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from . import abi

TCPDUMP_MAGIC = 0xA1B2C3D4
KUZNETZOV_MAGIC = 0xA1B2CD34
NSEC_MAGIC = 0xA1B23C4D
MAX_RECORD = 256 * 1024


@dataclass
class PacketBatch:
    """Packets stored back to back: packet i is data[offsets[i] : offsets[i] + caplens[i]]."""

    data: np.ndarray                 # uint8
    offsets: np.ndarray              # uint64
    caplens: np.ndarray              # uint32
    linktype: int = abi.LINKTYPE_ETHERNET
    timestamps_ns: np.ndarray | None = None
    frame_lens: np.ndarray | None = None
    meta: dict = field(default_factory=dict)

    @property
    def n(self) -> int:
        return int(self.caplens.shape[0])

    def packet(self, i: int) -> bytes:
        o = int(self.offsets[i])
        return self.data[o:o + int(self.caplens[i])].tobytes()

    def wire_bytes(self) -> int:
        return int(self.caplens.sum(dtype=np.uint64))

    def c_batch(self) -> abi.Batch:
        return abi.Batch(self.data.ctypes.data, self.offsets.ctypes.data, self.caplens.ctypes.data,
                         int(self.data.nbytes), self.n, self.linktype, 0)

    def slice(self, start: int, stop: int) -> "PacketBatch":
        """Packets [start, stop) repacked contiguously from offset 0."""
        offs = self.offsets[start:stop]
        caps = self.caplens[start:stop]
        if len(caps) == 0:
            return PacketBatch(np.zeros(1, np.uint8), offs.copy(), caps.copy(), self.linktype)
        lo = int(offs[0])
        hi = int(offs[-1]) + int(caps[-1])
        contiguous = bool(np.all(offs[1:] == offs[:-1] + caps[:-1]))
        if contiguous:
            data = self.data[lo:hi].copy()
            return PacketBatch(data, (offs - lo).astype(np.uint64), caps.copy(), self.linktype)
        return from_packets([self.packet(i) for i in range(start, stop)], self.linktype)


def from_packets(packets: list[bytes], linktype: int = abi.LINKTYPE_ETHERNET) -> PacketBatch:
    caps = np.array([len(p) for p in packets], dtype=np.uint32)
    offs = np.zeros(len(packets), dtype=np.uint64)
    if len(packets) > 1:
        offs[1:] = np.cumsum(caps[:-1], dtype=np.uint64)
    data = np.frombuffer(b"".join(packets) + b"\0", dtype=np.uint8).copy()
    return PacketBatch(data, offs, caps, linktype)


def concat(batches: list[PacketBatch]) -> PacketBatch:
    lt = {b.linktype for b in batches}
    if len(lt) != 1:
        raise ValueError("batches with different link types")
    pk = [b.packet(i) for b in batches for i in range(b.n)]
    return from_packets(pk, lt.pop())


def read_pcap(path: str | Path, max_packets: int | None = None) -> PacketBatch:
    raw = Path(path).read_bytes()
    if len(raw) < 24:
        raise ValueError(f"{path}: no pcap header")
    magic = struct.unpack("<I", raw[:4])[0]
    endian = "<"
    if magic in (TCPDUMP_MAGIC, KUZNETZOV_MAGIC, NSEC_MAGIC):
        pass
    else:
        magic = struct.unpack(">I", raw[:4])[0]
        if magic not in (TCPDUMP_MAGIC, KUZNETZOV_MAGIC, NSEC_MAGIC):
            raise ValueError(f"{path}: not a pcap file")
        endian = ">"
    nsec = magic == NSEC_MAGIC
    _, _, _, _, snaplen, linktype = struct.unpack(endian + "HHiIII", raw[4:24])
    linktype &= 0x0FFFFFFF
    pos = 24
    rec_hdr = 24 if magic == KUZNETZOV_MAGIC else 16
    chunks, caps, ts, flens = [], [], [], []
    limit = max_packets if max_packets is not None else 1 << 62
    while pos + rec_hdr <= len(raw) and len(caps) < limit:
        sec, sub, cap, flen = struct.unpack(endian + "IIII", raw[pos:pos + 16])
        pos += rec_hdr
        if cap > flen or cap > MAX_RECORD:
            break
        if sub >= (1_000_000_000 if nsec else 1_000_000):
            break
        keep = min(cap, snaplen) if snaplen else cap
        if pos + cap > len(raw):
            break
        chunks.append(raw[pos:pos + keep])
        pos += cap
        caps.append(keep)
        ts.append(sec * 1_000_000_000 + (sub if nsec else sub * 1000))
        flens.append(flen)
    b = from_packets(chunks, linktype)
    b.timestamps_ns = np.array(ts, dtype=np.uint64)
    b.frame_lens = np.array(flens, dtype=np.uint32)
    b.meta["source"] = str(path)
    return b


def write_pcap(path: str | Path, batch: PacketBatch, snaplen: int = 262144) -> None:
    out = [struct.pack("<IHHiIII", TCPDUMP_MAGIC, 2, 4, 0, 0, snaplen, batch.linktype)]
    ts = batch.timestamps_ns if batch.timestamps_ns is not None else np.zeros(batch.n, np.uint64)
    for i in range(batch.n):
        p = batch.packet(i)
        t = int(ts[i])
        flen = int(batch.frame_lens[i]) if batch.frame_lens is not None else len(p)
        out.append(struct.pack("<IIII", t // 1_000_000_000, (t % 1_000_000_000) // 1000, len(p), flen))
        out.append(p)
    Path(path).write_bytes(b"".join(out))


def read_hex_dat(path: str | Path) -> bytes:
    """One packet per file as hex text (the reference's Tests/Packet++Test/PacketExamples/*.dat)."""
    txt = "".join(Path(path).read_text().split())
    return bytes.fromhex(txt)
