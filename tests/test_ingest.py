"""Native pcap ingest (pcppx_pcap_*, csrc/pcppx_pcap.cpp) against the Python reader (pcap.read_pcap),
both following PcapFileReaderDevice (Pcap++/src/PcapFileDevice.cpp): magic variants, record checks that
end the stream, snapshot-length truncation, and batching by packet count and buffer size. Host only."""
from __future__ import annotations

import struct

import numpy as np
import pytest

from conftest import golden_files, load_golden
from pcapplusplus_amd import abi, synth
from pcapplusplus_amd.pcap import read_pcap, write_pcap


def native_read_all(path, max_packets=777, data_cap=1 << 20):
    from pcapplusplus_amd.engine import PcapReader

    pk, ts = [], []
    with PcapReader(path) as r:
        lt = r.linktype
        while True:
            b = r.read_batch(max_packets, data_cap)
            if b.n == 0:
                break
            pk += [b.packet(i) for i in range(b.n)]
            ts.append(b.timestamps_ns)
    return lt, pk, (np.concatenate(ts) if ts else np.zeros(0, np.uint64))


def py_read_all(path):
    b = read_pcap(path)
    return b.linktype, [b.packet(i) for i in range(b.n)], b.timestamps_ns


def write_variant(path, packets, magic=0xA1B2C3D4, endian="<", snaplen=262144, linktype=1, rec_extra=0,
                  caplen_fn=None, sub_fn=None):
    out = [struct.pack(endian + "IHHiIII", magic, 2, 4, 0, 0, snaplen, linktype)]
    for i, p in enumerate(packets):
        cap = len(p) if caplen_fn is None else caplen_fn(i, p)
        sub = (i * 37) % 1000 if sub_fn is None else sub_fn(i)
        out.append(struct.pack(endian + "IIII", 1700000000 + i, sub, cap, len(p)))
        out.append(b"\0" * rec_extra)
        out.append(p)
    path.write_bytes(b"".join(out))


def sample_packets():
    b = synth.config(3, 3000)
    return [b.packet(i) for i in range(b.n)]


@pytest.mark.parametrize("magic,endian,extra", [
    (0xA1B2C3D4, "<", 0), (0xA1B2C3D4, ">", 0),      # usec, native and swapped
    (0xA1B23C4D, "<", 0), (0xA1B23C4D, ">", 0),      # nsec
    (0xA1B2CD34, "<", 8), (0xA1B2CD34, ">", 8),      # Kuznetzov: 24-B record headers
], ids=["usec", "usec-swapped", "nsec", "nsec-swapped", "kuz", "kuz-swapped"])
def test_magic_variants(tmp_path, magic, endian, extra):
    pk = sample_packets()
    f = tmp_path / "v.pcap"
    write_variant(f, pk, magic, endian, rec_extra=extra)
    lt, got, ts = native_read_all(f)
    lt2, want, ts2 = py_read_all(f)
    assert lt == lt2 == 1
    assert got == want == pk
    assert np.array_equal(ts, ts2)


@pytest.mark.parametrize("path", [p for p in golden_files() if p.stem.startswith("pcap_")], ids=lambda p: p.stem)
def test_fixture_roundtrip(tmp_path, path):
    batch, _ = load_golden(path)
    f = tmp_path / "g.pcap"
    write_pcap(f, batch)
    lt, got, _ = native_read_all(f, max_packets=129, data_cap=70000)
    assert lt == batch.linktype & 0x0FFFFFFF
    assert got == [batch.packet(i) for i in range(batch.n)]


def test_stream_end_rules(tmp_path):
    pk = sample_packets()[:200]
    f = tmp_path / "bad.pcap"
    # caplen > frame length at record 50 ends the stream there
    write_variant(f, pk, caplen_fn=lambda i, p: len(p) + (1 if i == 50 else 0))
    assert native_read_all(f)[1] == py_read_all(f)[1]
    # out-of-range microseconds at record 70
    write_variant(f, pk, sub_fn=lambda i: 1_000_000 if i == 70 else 5)
    got = native_read_all(f)[1]
    assert got == py_read_all(f)[1] == pk[:70]
    # truncated final record
    write_variant(f, pk)
    f.write_bytes(f.read_bytes()[:-7])
    got = native_read_all(f)[1]
    assert got == py_read_all(f)[1] == pk[:-1]


def test_snaplen_truncation(tmp_path):
    pk = sample_packets()[:500]
    f = tmp_path / "snap.pcap"
    write_variant(f, pk, snaplen=96)
    got = native_read_all(f)[1]
    assert got == py_read_all(f)[1] == [p[:96] for p in pk]


def test_buffer_limits(tmp_path):
    from pcapplusplus_amd.engine import PcapReader

    pk = sample_packets()[:100]
    f = tmp_path / "buf.pcap"
    write_variant(f, pk)
    with PcapReader(f) as r:
        with pytest.raises(RuntimeError):
            r.read_batch(10, data_cap=16)  # one record does not fit
    with PcapReader(f) as r:
        b = r.read_batch(1000, data_cap=4096)
        assert 0 < b.n < 100 and b.wire_bytes() <= 4096
        assert [b.packet(i) for i in range(b.n)] == pk[:b.n]


def test_rejects_non_pcap(tmp_path):
    from pcapplusplus_amd.engine import PcapReader

    f = tmp_path / "x.pcap"
    f.write_bytes(b"\x0a\x0d\x0d\x0a" + b"\0" * 60)  # pcapng section header: not this reader's format
    with pytest.raises(RuntimeError):
        PcapReader(f)
    with pytest.raises(RuntimeError):
        PcapReader(tmp_path / "missing.pcap")
