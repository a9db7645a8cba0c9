"""Crafted and mutated capture files for the ingest parity tests (host only).

Every case is a (name, bytes) pair generated from a seed, so tests/golden/ingest/expected.npz (written by
tools/make_golden_ingest.py from the REAL reference readers, PcapFileReaderDevice / PcapNgFileReaderDevice
over LightPcapNg) can be re-checked without /root/reference. The crafted cases walk the reference's rules:
Pcap++/src/PcapFileDevice.cpp:53-87 (magics, headers), :707-768 (open checks), :799-886 (record checks);
3rdParty/LightPcapNg/LightPcapNg/src/light_pcapng.c:36-93,101-211,341-423 and light_pcapng_ext.c:43-55,
140-167,380-479 (pcapng blocks, interfaces, if_tsresol, EPB/SPB).
"""
from __future__ import annotations

import random
import struct

import numpy as np

from pcapplusplus_amd import synth


def sample_packets(n: int = 40, seed: int = 7) -> list[bytes]:
    b = synth.imix(n, seed)
    return [b.packet(i) for i in range(b.n)]


# ---------------------------------------------------------------- pcap
def pcap_file(packets, magic=0xA1B2C3D4, endian="<", vmaj=2, snaplen=262144, linktype=1, caplen_fn=None,
              len_fn=None, sub_fn=None, rec_extra=b"") -> bytes:
    out = [struct.pack(endian + "IHHiIII", magic, vmaj, 4, 0, 0, snaplen, linktype)]
    for i, p in enumerate(packets):
        cap = len(p) if caplen_fn is None else caplen_fn(i, p)
        ln = len(p) if len_fn is None else len_fn(i, p)
        sub = (i * 37) % 1000 if sub_fn is None else sub_fn(i)
        out.append(struct.pack(endian + "IIII", 1700000000 + i, sub, cap, ln))
        out.append(rec_extra)
        out.append(p)
    return b"".join(out)


def pcap_cases() -> list[tuple[str, bytes]]:
    pk = sample_packets(40)
    c = []
    for magic, tag in ((0xA1B2C3D4, "usec"), (0xA1B23C4D, "nsec"), (0xA1B2CD34, "kuz")):
        for endian, et in (("<", "le"), (">", "be")):
            c.append((f"pcap_{tag}_{et}", pcap_file(pk, magic, endian)))
            c.append((f"pcap_{tag}_{et}_rec24", pcap_file(pk, magic, endian, rec_extra=b"\x11" * 8)))
    c.append(("pcap_nsec_sub_max", pcap_file(pk, 0xA1B23C4D, sub_fn=lambda i: 999_999_999 if i < 5 else 1_000_000_000)))
    c.append(("pcap_usec_sub_max", pcap_file(pk, sub_fn=lambda i: 999_999 if i < 7 else 1_000_000)))
    for v in (0, 1, 2, 3, 543, 544):
        c.append((f"pcap_vmaj{v}", pcap_file(pk[:3], vmaj=v)))
    for s in (0, 1, 60, 96, 1 << 20, (1 << 20) + 1, 0xFFFFFFFF):
        c.append((f"pcap_snap{s}", pcap_file(pk, snaplen=s)))
    for lt in (0, 1, 2, 12, 101, 113, 228, 276, 277, 0xFFFF, 0x08000001, 0x10000001):
        c.append((f"pcap_lt{lt}", pcap_file(pk[:4], linktype=lt)))
    c.append(("pcap_cap_gt_len", pcap_file(pk, caplen_fn=lambda i, p: len(p), len_fn=lambda i, p: len(p) - (i == 9))))
    big = [bytes(range(256)) * 1100]  # 281,600 B > 256 KiB
    c.append(("pcap_cap_256k", pcap_file(pk[:3] + big + pk[3:6], snaplen=1 << 20)))
    c.append(("pcap_cap_zero", pcap_file([b""] + pk[:5] + [b""])))
    c.append(("pcap_empty", pcap_file([])))
    f = pcap_file(pk)
    for cut in (1, 4, 15, 16, 17, 23, 24, 25, 39, 40, 41):
        c.append((f"pcap_cut{cut}", f[:cut] if cut <= 24 else f[:-cut]))
    # snaplen truncation with the skipped tail running past the end of the file (delivered: ignore() only sets eof)
    g = pcap_file(pk[:6], snaplen=60)
    c.append(("pcap_snap_tail_cut", g[:-(len(pk[5]) - 70)] if len(pk[5]) > 80 else g[:-3]))
    c.append(("pcap_short_header", b"\xd4\xc3\xb2\xa1" + b"\x02\x00\x04\x00" + b"\0" * 10))
    c.append(("pcap_bad_magic", b"\xd4\xc3\xb2\xa2" + f[4:]))
    return c


# ---------------------------------------------------------------- pcapng
def block(btype: int, body: bytes, total: int | None = None, trailer: int | None = None) -> bytes:
    pad = (-len(body)) % 4
    t = 12 + len(body) + pad if total is None else total
    return struct.pack("<II", btype, t) + body + b"\0" * pad + struct.pack("<I", t if trailer is None else trailer)


def opt(code: int, data: bytes) -> bytes:
    return struct.pack("<HH", code, len(data)) + data + b"\0" * ((-len(data)) % 4)


END = struct.pack("<HH", 0, 0)


def shb(opts: bytes = b"") -> bytes:
    return block(0x0A0D0D0A, struct.pack("<IHHq", 0x1A2B3C4D, 1, 0, -1) + opts)


def idb(linktype: int = 1, tsresol: int | None = None, snap: int = 0, extra_opts: bytes = b"") -> bytes:
    o = extra_opts
    if tsresol is not None:
        o += opt(9, bytes([tsresol]))
    if o:
        o += END
    return block(1, struct.pack("<HHI", linktype, 0, snap) + o)


def epb(data: bytes, ifid: int = 0, ts: int = 1_700_000_000_123_456, cap: int | None = None, orig: int | None = None,
        opts: bytes = b"") -> bytes:
    c = len(data) if cap is None else cap
    o = len(data) if orig is None else orig
    body = struct.pack("<IIIII", ifid, ts >> 32, ts & 0xFFFFFFFF, c, o) + data + b"\0" * ((-len(data)) % 4) + opts
    return block(6, body)


def spb(data: bytes, orig: int | None = None) -> bytes:
    return block(3, struct.pack("<I", len(data) if orig is None else orig) + data)


def pcapng_cases() -> list[tuple[str, bytes]]:
    pk = sample_packets(24, seed=11)
    c = []
    base = shb() + idb(1) + b"".join(epb(p, ts=1_700_000_000_000_000 + 1000 * i) for i, p in enumerate(pk))
    c.append(("ng_basic", base))
    c.append(("ng_shb_opts", shb(opt(2, b"hw") + opt(3, b"linux") + opt(4, b"app") + END) + base[len(shb()):]))
    for r in (0, 3, 6, 9, 10, 12, 19, 128, 128 + 10, 128 + 31, 128 + 32, 128 + 40, 255):
        ts = 1_700_000_000 * 10 ** min(r, 9) + 12345 if r < 128 else (1_700_000_000 << min(r - 128, 20)) + 77
        c.append((f"ng_tsresol{r}", shb() + idb(1, r) + b"".join(epb(p, ts=ts + i) for i, p in enumerate(pk[:4]))))
    c.append(("ng_tsresol_after_other_opt", shb() + idb(1, None, extra_opts=opt(2, b"eth0") + opt(9, b"\x09"))
              + epb(pk[0], ts=1_700_000_000_000_000_123)))
    c.append(("ng_ts_zero_secs", shb() + idb(1) + epb(pk[0], ts=999_999) + epb(pk[1], ts=1_000_000)))
    c.append(("ng_ts_huge", shb() + idb(1, 0) + epb(pk[0], ts=(1 << 64) - 1) + epb(pk[1], ts=18446744073 + 1)))
    two = shb() + idb(1) + idb(113, 9) + idb(101)
    c.append(("ng_multi_if", two + b"".join(epb(p, ifid=i % 4, ts=(1 + i) * 10 ** 15) for i, p in enumerate(pk))))
    c.append(("ng_if_late", shb() + idb(1) + epb(pk[0]) + idb(228) + epb(pk[1], ifid=1) + epb(pk[2], ifid=0)))
    c.append(("ng_many_if", shb() + b"".join(idb(1 + (k % 3)) for k in range(40))
              + b"".join(epb(p, ifid=(7 * i) % 40) for i, p in enumerate(pk))))
    c.append(("ng_two_sections", base + shb() + idb(101) + b"".join(epb(p, ifid=1) for p in pk[:5])))
    c.append(("ng_unknown_blocks", shb() + block(0x0BAD, b"x" * 13) + idb(1) + block(5, b"\0" * 28)
              + block(4, b"\1\0\4\0abcd\0\0\0\0") + epb(pk[0]) + block(0x40000BAD, b"y" * 8) + epb(pk[1])))
    c.append(("ng_epb_cap_gt_block", shb() + idb(1) + epb(pk[0], cap=len(pk[0]) + 50) + epb(pk[1])))
    c.append(("ng_epb_cap_zero", shb() + idb(1) + epb(b"") + epb(pk[1], cap=0)))
    c.append(("ng_epb_orig_small", shb() + idb(1) + epb(pk[0], orig=3) + epb(pk[1], orig=0xFFFFFFFF)))
    c.append(("ng_epb_opts", shb() + idb(1) + epb(pk[0], opts=opt(1, b"a comment") + END) + epb(pk[1])))
    c.append(("ng_spb", shb() + idb(113) + spb(pk[0]) + spb(pk[1], orig=len(pk[1]) - 5) + epb(pk[2])))
    c.append(("ng_no_shb", idb(1) + epb(pk[0])))
    c.append(("ng_trailer_mismatch", shb() + idb(1) + epb(pk[0]) + block(6, epb(pk[1])[8:-4], trailer=99) + epb(pk[2])))
    c.append(("ng_shb_trailer_mismatch", block(0x0A0D0D0A, struct.pack("<IHHq", 0x1A2B3C4D, 1, 0, -1), trailer=7)
              + idb(1) + epb(pk[0])))
    c.append(("ng_only_shb", shb()))
    c.append(("ng_no_packets", shb() + idb(1) + idb(113)))
    c.append(("ng_empty_idb_opts", shb() + block(1, struct.pack("<HHI", 1, 0, 0) + END) + epb(pk[0])))
    c.append(("ng_bad_opt_len", shb() + block(1, struct.pack("<HHI", 1, 0, 0) + struct.pack("<HH", 9, 200) + b"\x09\0\0\0")
              + epb(pk[0], ts=5 * 10 ** 6)))
    c.append(("ng_zero_len_opt", shb() + block(1, struct.pack("<HHI", 1, 0, 0) + struct.pack("<HH", 2, 0)
                                                 + opt(9, b"\x03") + END) + epb(pk[0], ts=5 * 10 ** 6)))
    f = base
    for cut in (4, 8, 12, 27, 28, 40, 50, 60, 61, 100):
        c.append((f"ng_cut{cut}", f[:cut] if cut <= 28 else f[:-cut]))
    return c


# ---------------------------------------------------------------- mutations
def mutate(data: bytes, rng: random.Random) -> bytes:
    """One seeded structural mutation: header-word overwrites, byte flips, truncation, splices."""
    b = bytearray(data)
    if not b:
        return bytes(b)
    k = rng.randrange(7)
    if k == 0:  # overwrite a 32-bit word near a record/block boundary with an interesting value
        pos = rng.randrange(0, max(1, min(len(b) - 4, 4096))) & ~3
        v = rng.choice([0, 1, 4, 8, 11, 12, 13, 16, 20, 28, 31, 32, 33, 0xFFFF, 0x10000, 0x40000, 0x40001,
                        0x7FFFFFFF, 0xFFFFFFFF, rng.randrange(1 << 32)])
        b[pos:pos + 4] = struct.pack("<I", v)
    elif k == 1:  # random byte flips in the first 512 bytes
        for _ in range(rng.randrange(1, 6)):
            i = rng.randrange(min(len(b), 512))
            b[i] ^= 1 << rng.randrange(8)
    elif k == 2:  # truncate anywhere
        b = b[: rng.randrange(len(b))]
    elif k == 3:  # duplicate a slice (repeated records / blocks)
        i = rng.randrange(len(b))
        j = min(len(b), i + rng.randrange(1, 200))
        b[i:i] = b[i:j]
    elif k == 4:  # delete a slice
        i = rng.randrange(len(b))
        del b[i:i + rng.randrange(1, 64)]
    elif k == 5:  # 16-bit overwrites (pcap version, pcapng option code/length, IDB link type)
        pos = rng.randrange(0, max(1, min(len(b) - 2, 2048))) & ~1
        b[pos:pos + 2] = struct.pack("<H", rng.choice([0, 1, 2, 3, 9, 0x80, 0xFF, 0xFFFF, rng.randrange(1 << 16)]))
    else:  # random bytes over a window
        i = rng.randrange(len(b))
        for t in range(i, min(len(b), i + rng.randrange(1, 32))):
            b[t] = rng.randrange(256)
    return bytes(b)


def mutation_cases(seeds: list[tuple[str, bytes]], per_seed: int, seed: int = 2024) -> list[tuple[str, bytes]]:
    rng = random.Random(seed)
    out = []
    for name, data in seeds:
        for k in range(per_seed):
            d = data
            for _ in range(rng.randrange(1, 4)):
                d = mutate(d, rng)
            out.append((f"mut_{name}_{k}", d))
    return out


def reference_undefined(data: bytes) -> str | None:
    """Why the reference's reading of this capture is undefined behaviour (it reads past its heap buffer or
    an uninitialised value), or None. Walks the pcapng blocks as light_get_next_packet would, up to where
    the stream ends: a block total length below 12 (light_pcapng.c:393 wraps bytesToRead), an IDB body
    shorter than link type + snaplen (:135-140), an EPB body shorter than its five fields (:155-159), an
    SPB shorter than its length field or whose original length exceeds its body (:200-206 +
    PcapFileDevice.cpp:1214-1215), or an SPB before any interface (light_pcapng_ext.c:462-463 leaves
    data_link unset). pcap files have no such cases."""
    if len(data) < 4 or struct.unpack_from("<I", data)[0] != 0x0A0D0D0A:
        return None

    def block_at(p):
        if len(data) - p < 8:
            return None
        t, n = struct.unpack_from("<II", data, p)
        if n < 12:
            return "ub", "block total length below 12"
        if len(data) - p < n or struct.unpack_from("<I", data, p + n - 4)[0] != n:
            return None
        return t, n

    r = block_at(0)
    if r is None or r[0] == "ub":
        return None if r is None else r[1]
    if r[0] != 0x0A0D0D0A:
        return None
    p, n_if = r[1], 0
    while True:
        r = block_at(p)
        if r is None:
            return None
        if r[0] == "ub":
            return r[1]
        t, n = r
        if t == 1:
            if n < 20:
                return "short interface block"
            n_if += 1
        elif t == 6 and n < 32:
            return "short enhanced packet block"
        elif t == 3:
            if n < 16:
                return "short simple packet block"
            if n_if == 0:
                return "simple packet block before any interface"
            if struct.unpack_from("<I", data, p + 8)[0] > n - 16:
                return "simple packet block original length beyond its body"
        p += n


def crafted_cases() -> list[tuple[str, bytes]]:
    return pcap_cases() + pcapng_cases()


def digest(packets: list[bytes]) -> np.ndarray:
    """8-byte BLAKE2b digest per packet (the golden file stores digests, not the bytes)."""
    import hashlib

    return np.array([int.from_bytes(hashlib.blake2b(p, digest_size=8).digest(), "little") for p in packets],
                    dtype=np.uint64)
