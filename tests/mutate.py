"""Seeded adversarial packet generators for parity tests (test helper).

Mutations of real fixture packets (bit flips concentrated in the first 80 bytes, truncation, random
re-slicing) plus hand-built deep/odd stacks: QinQ, MPLS stacks, GRE with every flag combination,
IPv6 extension chains that run past the 128-byte staging window, odd lengths, tiny packets.
"""
from __future__ import annotations

import struct

import numpy as np

from pcapplusplus_amd.pcap import PacketBatch, from_packets


def mutate(packets: list[bytes], n: int, seed: int) -> list[bytes]:
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        p = bytearray(packets[int(rng.integers(len(packets)))])
        op = int(rng.integers(6))
        if op in (0, 1, 2) and len(p):
            for _ in range(int(rng.integers(1, 4))):
                j = int(rng.integers(min(len(p), 80)))
                p[j] ^= 1 << int(rng.integers(8))
        elif op == 3 and len(p) > 1:
            p = p[: int(rng.integers(1, len(p)))]
        elif op == 4 and len(p) > 20:
            j = int(rng.integers(14, min(len(p), 70)))
            p[j] = int(rng.integers(256))
            p[j - 1] = int(rng.integers(256))
        out.append(bytes(p))
    return out


def _eth(et: int) -> bytes:
    return bytes.fromhex("001122334455") + bytes.fromhex("66778899aabb") + struct.pack(">H", et)


def _ipv4(proto: int, payload_len: int, ihl: int = 5, frag: int = 0x4000) -> bytes:
    h = bytearray(ihl * 4)
    h[0] = 0x40 | ihl
    struct.pack_into(">HHHBB", h, 2, ihl * 4 + payload_len, 7, frag, 64, proto)
    h[12:16] = bytes([10, 1, 2, 3])
    h[16:20] = bytes([192, 168, 9, 1])
    return bytes(h)


def _ipv6(nh: int, payload_len: int) -> bytes:
    h = bytearray(40)
    h[0] = 0x60
    struct.pack_into(">HBB", h, 4, payload_len, nh, 64)
    h[8:24] = bytes(range(16))
    h[24:40] = bytes(range(100, 116))
    return bytes(h)


def _udp(sport: int, dport: int, payload: bytes) -> bytes:
    return struct.pack(">HHHH", sport, dport, 8 + len(payload), 0x1234) + payload


def _tcp(sport: int, dport: int, payload: bytes, doff: int = 5) -> bytes:
    h = bytearray(doff * 4)
    struct.pack_into(">HHIIBBHHH", h, 0, sport, dport, 1, 2, doff << 4, 0x18, 1000, 0xABCD, 0)
    return bytes(h) + payload


def crafted(seed: int = 7) -> list[bytes]:
    """Deep and odd layer stacks covering every in-scope rule and the LDS-window fallback."""
    rng = np.random.default_rng(seed)
    pay = lambda k: rng.bytes(k)  # noqa: E731
    pk = []
    l4s = [_udp(40000, 50000, pay(33)), _tcp(40001, 50001, pay(101)), _tcp(40002, 50002, pay(7), doff=15)]
    # QinQ + MPLS stacks + IPv4/IPv6
    for l4 in l4s:
        proto = 17 if len(l4) and l4[12] == 0 and False else (6 if l4 is not l4s[0] else 17)
        ip4 = _ipv4(proto, len(l4))
        ip6 = _ipv6(proto, len(l4))
        vl = lambda et: struct.pack(">HH", 0x0123, et)  # noqa: E731
        pk.append(_eth(0x88A8) + vl(0x8100) + vl(0x0800) + ip4 + l4)
        pk.append(_eth(0x8100) + vl(0x8100) + vl(0x8100) + vl(0x86DD) + ip6 + l4)
        for labels in (1, 2, 3, 5):
            m = b"".join(struct.pack(">I", (100 + k) << 12 | (1 if k == labels - 1 else 0) << 8 | 64)
                         for k in range(labels))
            pk.append(_eth(0x8847) + m + ip4 + l4)
            pk.append(_eth(0x8847) + m + ip6 + l4)
        # GRE v0 with every C/R/K/S combination, over IPv4 and IPv6, carrying IPv4 / IPv6 / Eth / VLAN / MPLS
        for flags in range(16):
            b0 = ((flags & 1) << 7) | ((flags & 2) << 5) | ((flags & 4) << 3) | ((flags & 8) << 1)
            opt = b"\xaa" * (4 * (bool(flags & 3) + bool(flags & 4) + bool(flags & 8)))
            for inner_et, inner in ((0x0800, ip4 + l4), (0x86DD, ip6 + l4), (0x6558, _eth(0x0800) + ip4 + l4),
                                    (0x8100, struct.pack(">HH", 5, 0x0800) + ip4 + l4),
                                    (0x8847, struct.pack(">I", 200 << 12 | 1 << 8 | 9) + ip6 + l4)):
                gre = bytes([b0, 0]) + struct.pack(">H", inner_et) + opt + inner
                pk.append(_eth(0x0800) + _ipv4(47, len(gre)) + gre)
                pk.append(_eth(0x86DD) + _ipv6(47, len(gre)) + gre)
        # GREv1 (PPTP) with PPP carrying IPv4/IPv6
        for ppp_proto, inner in ((0x21, ip4 + l4), (0x57, ip6 + l4), (0x99, pay(20))):
            ppp = bytes([0xFF, 0x03]) + struct.pack(">H", ppp_proto) + inner
            gre1 = bytes([0x30, 0x81]) + struct.pack(">HHH", 0x880B, len(ppp), 7) + b"\x00" * 8 + ppp
            pk.append(_eth(0x0800) + _ipv4(47, len(gre1)) + gre1)
        # IPv6 extension chains, some longer than the 128-B staging window
        for chain in ((0,), (0, 60), (43, 60), (0, 43, 60, 60), (44,), (0, 44), (51,), (60, 51)):
            exts = b""
            nxt = [*chain[1:], 6 if l4 is not l4s[0] else 17]
            for t, nh in zip(chain, nxt):
                if t == 51:
                    e = bytes([nh, 4]) + b"\x00" * 22
                elif t == 44:
                    e = bytes([nh, 0]) + b"\x00\x01" + b"\x00" * 4
                else:
                    hl = int(rng.integers(0, 6))
                    e = bytes([nh, hl]) + b"\x01" * (8 * (hl + 1) - 2)
                exts += e
            body = exts + l4
            pk.append(_eth(0x86DD) + _ipv6(chain[0], len(body)) + body)
        # IPv4 options, IPIP, 6in4, fragments, TSO (totalLength 0), padding/trailers
        for ihl in (5, 6, 10, 15):
            pk.append(_eth(0x0800) + _ipv4(6 if l4 is not l4s[0] else 17, len(l4), ihl) + l4)
        pk.append(_eth(0x0800) + _ipv4(4, 20 + len(l4)) + _ipv4(17 if l4 is l4s[0] else 6, len(l4)) + l4)
        pk.append(_eth(0x0800) + _ipv4(41, 40 + len(l4)) + _ipv6(17 if l4 is l4s[0] else 6, len(l4)) + l4)
        pk.append(_eth(0x0800) + _ipv4(6, len(l4), frag=0x2000) + l4)
        pk.append(_eth(0x0800) + _ipv4(6, len(l4), frag=0x0010) + l4)
        tso = bytearray(_ipv4(6, len(l4)))
        tso[2:4] = b"\x00\x00"
        pk.append(_eth(0x0800) + bytes(tso) + l4)
        pk.append(_eth(0x0800) + _ipv4(17 if l4 is l4s[0] else 6, len(l4)) + l4 + b"\x00" * 18)
        pk.append(_eth(0x86DD) + _ipv6(17 if l4 is l4s[0] else 6, len(l4)) + l4 + b"\xee" * 5)
    # L2 odds: 802.3 + LLC (+STP), VLAN -> LLC, unknown ethertypes, runts
    pk.append(bytes(12) + struct.pack(">H", 0x26) + bytes([0xAA, 0xAA, 0x03]) + pay(40))
    pk.append(bytes(12) + struct.pack(">H", 0x26) + bytes([0x42, 0x42, 0x03]) + pay(40))
    pk.append(bytes(12) + struct.pack(">H", 0x26) + bytes([0xFF, 0xFF, 0x03]) + pay(40))
    pk.append(_eth(0x8100) + struct.pack(">HH", 3, 0x0040) + bytes([0xAA, 0xAA, 0x03]) + pay(30))
    pk.append(_eth(0x0700) + pay(30))
    pk.append(_eth(0x9000) + pay(30))
    for k in range(0, 40):
        pk.append(_eth(0x0800)[: min(k, 14)] + _ipv4(6, 20)[: max(0, k - 14)])
    pk.append(_eth(0x8100) + b"\x00\x01")                       # unchecked VLAN shorter than its header
    pk.append(_eth(0x8847) + b"\x00\x00\x00")                   # MPLS shorter than 5
    pk.append(_eth(0x8100) * 1 + b"".join(struct.pack(">HH", 1, 0x8100) for _ in range(20)) + pay(10))
    # L7 triggers and SIP heuristic (flagged)
    pk.append(_eth(0x0800) + _ipv4(6, 20 + 10) + _tcp(50000, 80, b"GET / HTTP"))
    pk.append(_eth(0x0800) + _ipv4(17, 8 + 12) + _udp(50000, 50001, b"INVITE sip:x"))
    pk.append(_eth(0x0800) + _ipv4(17, 8 + 12) + _udp(53, 50001, pay(12)))
    pk.append(_eth(0x0806) + pay(28))
    pk.append(_eth(0x0800) + _ipv4(1, 8) + pay(8))
    # ICMP (IcmpLayer.cpp:562-620, IcmpLayer.h:619-660): every type 0-20 at and around its message size, error
    # messages quoting an IPv4 header (+ TCP / UDP, cut short), router advertisements with counts past the data,
    # behind a VLAN, GRE, an IPv4 fragment and IPv6 (next header 1 is no ICMP there), padded for a trailer
    inner = [b"", _ipv4(6, 20)[:12], _ipv4(6, 8) + _tcp(1, 2, b"")[:8], _ipv4(17, 8) + _udp(53, 9, b""),
             _ipv4(1, 8) + bytes([8, 0, 0, 0]) + pay(4), _ipv4(6, 40) + _tcp(80, 3, pay(20))]
    for t in range(21):
        for n in (3, 4, 7, 8, 11, 12, 19, 20, 24, 40):
            body = bytes([t, 0, 0, 0]) + pay(max(0, n - 4))
            body = body[:n]
            pk.append(_eth(0x0800) + _ipv4(1, len(body)) + body)
        if t in (3, 4, 5, 11, 12):
            for inn in inner:
                body = bytes([t, 1, 0, 0]) + pay(4) + inn
                pk.append(_eth(0x0800) + _ipv4(1, len(body)) + body)
                pk.append(_eth(0x0800) + _ipv4(1, len(body)) + body + b"\x00" * 6)
    for cnt, extra in ((0, 0), (1, 8), (2, 8), (3, 30), (255, 16)):
        body = bytes([9, 0, 0, 0, cnt, 2, 0, 30]) + pay(extra)
        pk.append(_eth(0x0800) + _ipv4(1, len(body)) + body)
    echo = bytes([8, 0, 0, 0]) + pay(36)
    pk.append(_eth(0x8100) + struct.pack(">HH", 4, 0x0800) + _ipv4(1, len(echo)) + echo)
    gre = bytes([0, 0]) + struct.pack(">H", 0x0800) + _ipv4(1, len(echo)) + echo
    pk.append(_eth(0x0800) + _ipv4(47, len(gre)) + gre)
    pk.append(_eth(0x0800) + _ipv4(1, len(echo), frag=0x2000) + echo)
    pk.append(_eth(0x86DD) + _ipv6(1, len(echo)) + echo)
    pk.append(_eth(0x0800) + _ipv4(1, len(echo)) + echo + b"\xee" * 9)
    # tunnels over UDP (UdpLayer.cpp:103-131): VXLAN (VxlanLayer.cpp:50-58) and GTPv1 (GtpLayer.cpp:199-207,
    # 560-632) with inner stacks, extension chains, GTP-C lengths, and the port combinations that keep an earlier
    # dissector (DHCP, DNS, SIP, RADIUS) in front
    t4 = _tcp(1000, 2000, pay(10))
    in4 = _ipv4(6, len(t4)) + t4
    u53 = _udp(3000, 53, pay(20))
    in6 = _ipv6(17, len(u53)) + u53
    vx = bytes([8, 0, 0, 0, 0, 1, 2, 0])
    for inner in (_eth(0x0800) + in4, _eth(0x86DD) + in6, _eth(0x0800)[:13], bytes(12) + b"\x05\xdc" + pay(8), b"",
                  _eth(0x0800) + _ipv4(17, 16) + _udp(5, 4789, vx + _eth(0x0800) + in4)[:24], pay(3)):
        for v in (vx, vx[:7]):
            u = _udp(40000, 4789, v + inner)
            pk.append(_eth(0x0800) + _ipv4(17, len(u)) + u)
            pk.append(_eth(0x86DD) + _ipv6(17, len(u)) + u + b"\x00" * 3)
    u = _udp(4789, 40000, vx + _eth(0x0800) + in4)  # source port only: no VXLAN
    pk.append(_eth(0x0800) + _ipv4(17, len(u)) + u)

    def gtp(fl, mt, body, extra=b""):
        return bytes([fl, mt]) + struct.pack(">HI", len(extra) + len(body), 0x1234) + extra + body
    exts = [b"", bytes([1, 0x12, 0, 0]), bytes([1, 0x12, 0, 0x85]) + bytes([2, 1, 2, 3, 4, 5, 6, 0]),
            bytes([1, 0, 0, 0x85]), bytes([0, 9, 9, 9]), bytes([3, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 0]),
            bytes([9, 1, 2, 3]), bytes([1, 2, 3, 0x40]) + bytes([1, 2, 3, 0])]
    for fl in (0x30, 0x32, 0x34, 0x31, 0x36, 0x37, 0x20, 0x50, 0x10):
        for ext in exts:
            nt = ext[0] if False else (0x85 if ext else 0)
            extra = (b"\x00\x01\x00" + bytes([nt]) + ext) if fl & 7 else b""
            for body in (in4, in6, bytes([0x4f]) + in4[1:], bytes([0x44]) + in4[1:], in4[:19], pay(6), b""):
                g = gtp(fl, 0xFF, body, extra)
                u = _udp(2152, 2152, g)
                pk.append(_eth(0x0800) + _ipv4(17, len(u)) + u)
    for ports in ((2123, 40000), (40000, 2123), (2152, 53), (53, 2152), (2152, 5060), (1812, 2152), (67, 2152),
                  (2152, 4789), (2152, 40000)):
        for mt, ml in ((0xFF, None), (1, 4), (1, 400), (16, 0)):
            g = gtp(0x32, mt, in4, b"\x00\x01\x00\x00")
            if ml is not None:
                g = g[:2] + struct.pack(">H", ml) + g[4:]
            u = _udp(ports[0], ports[1], g)
            pk.append(_eth(0x0800) + _ipv4(17, len(u)) + u)
        u = _udp(ports[0], ports[1], gtp(0x30, 0xFF, in4)[:7])
        pk.append(_eth(0x0800) + _ipv4(17, len(u)) + u)
    return pk


def fragments(n: int, seed: int = 13) -> list[bytes]:
    """IP fragments and TCP segments for the reassembly front ends: IPv4 with every MF/offset shape, IHL
    larger than totalLength (malformed), IPv6 fragment headers first or behind other extensions (and
    twice), fragment headers cut by caplen, tunnels (IPv4 in IPv6, 6in4, GRE, VLAN/MPLS), TCP with every
    SYN/FIN/RST/ACK combination with and without payload, and UDP/ICMP around them."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        pay = rng.bytes(int(rng.integers(0, 60))) if rng.random() < 0.7 else b""
        flags = int(rng.choice([0x02, 0x12, 0x10, 0x18, 0x01, 0x11, 0x04, 0x14, 0x03, 0x07, 0x00]))
        l4k = int(rng.integers(4))
        if l4k == 0:
            l4, proto = _udp(40000 + int(rng.integers(1000)), 50000, pay), 17
        else:
            h = bytearray(_tcp(41000 + int(rng.integers(1000)), 51000, pay))
            h[13] = flags
            l4, proto = bytes(h), 6
        kind = int(rng.integers(8))
        if kind in (0, 1):  # IPv4, any MF/offset, sometimes an IHL past totalLength
            frag = int(rng.choice([0x0000, 0x4000, 0x2000, 0x2000 | int(rng.integers(1, 8192)),
                                   int(rng.integers(1, 8192))]))
            ihl = int(rng.choice([5, 5, 6, 15]))
            ip = bytearray(_ipv4(proto, len(l4), ihl, frag))
            ip[4:6] = rng.bytes(2)
            if rng.random() < 0.15:
                ip[2:4] = (ihl * 4 - 4 * int(rng.integers(1, 4))).to_bytes(2, "big")  # totalLength < IHL*4
            pk = _eth(0x0800) + bytes(ip) + l4
        elif kind in (2, 3, 4):  # IPv6 with a fragment header somewhere in its extension chain
            chain = [int(x) for x in rng.choice([0, 60, 43, 44], size=int(rng.integers(1, 4)))]
            if 44 not in chain and rng.random() < 0.8:
                chain.insert(int(rng.integers(len(chain) + 1)), 44)
            exts = b""
            nxt = [*chain[1:], proto]
            for t, nh in zip(chain, nxt):
                if t == 44:
                    off = int(rng.integers(0, 8192)) if rng.random() < 0.6 else 0
                    m = int(rng.integers(2))
                    exts += bytes([nh, 0]) + ((off << 3) | m).to_bytes(2, "big") + rng.bytes(4)
                else:
                    hl = int(rng.integers(0, 3))
                    exts += bytes([nh, hl]) + rng.bytes(8 * (hl + 1) - 2)
            body = exts + l4
            pk = _eth(0x86DD) + _ipv6(chain[0], len(body)) + body
            if rng.random() < 0.1:  # cut inside the extension chain
                pk = pk[: 54 + int(rng.integers(2, max(3, len(exts))))]
            elif rng.random() < 0.05:  # a leading fragment header cut by caplen (its fields past the packet)
                body = bytes([proto, 0]) + rng.bytes(6)
                pk = (_eth(0x86DD) + _ipv6(44, 8) + body)[: 54 + int(rng.integers(2, 8))]
        elif kind == 5:  # tunnels: IPv4 fragment inside IPv6, IPv6 fragment inside IPv4 (6in4), GRE, VLAN, MPLS
            inner4 = _ipv4(proto, len(l4), 5, int(rng.choice([0x2000, 0x0100, 0x4000])))
            inner6 = _ipv6(44, 8 + len(l4)) + bytes([proto, 0, 0, 9]) + rng.bytes(4) + l4
            t = int(rng.integers(5))
            if t == 0:
                pk = _eth(0x86DD) + _ipv6(4, len(inner4) + len(l4)) + inner4 + l4
            elif t == 1:
                pk = _eth(0x0800) + _ipv4(41, len(inner6)) + inner6
            elif t == 2:
                gre = bytes([0, 0]) + struct.pack(">H", 0x0800) + inner4 + l4
                pk = _eth(0x86DD) + _ipv6(47, len(gre)) + gre
            elif t == 3:
                pk = _eth(0x8100) + struct.pack(">HH", 7, 0x86DD) + inner6
            else:
                pk = _eth(0x8847) + struct.pack(">I", 100 << 12 | 1 << 8 | 64) + inner4 + l4
        elif kind == 6:  # ICMP / non-IP neighbours
            pk = [_eth(0x0800) + _ipv4(1, 8) + rng.bytes(8), _eth(0x0806) + rng.bytes(28),
                  _eth(0x9000) + rng.bytes(30)][int(rng.integers(3))]
        else:  # plain TCP/UDP over IPv4 or IPv6, sometimes padded
            ip = _ipv4(proto, len(l4)) if rng.random() < 0.5 else _ipv6(proto, len(l4))
            pk = _eth(0x0800 if len(ip) == 20 else 0x86DD) + ip + l4 + (b"\x00" * int(rng.integers(0, 20)))
        out.append(pk)
    return out


def as_batch(packets: list[bytes], gaps: bool = False, seed: int = 0) -> PacketBatch:
    """Pack packets; with gaps=True leave random gaps so packets start at every byte alignment."""
    if not gaps:
        return from_packets(packets)
    rng = np.random.default_rng(seed)
    offs, pos, chunks = [], 0, []
    for p in packets:
        g = int(rng.integers(0, 17))
        chunks.append(b"\xcc" * g)
        pos += g
        offs.append(pos)
        chunks.append(p)
        pos += len(p)
    data = np.frombuffer(b"".join(chunks) + b"\0" * 16, dtype=np.uint8).copy()
    return PacketBatch(data, np.array(offs, np.uint64), np.array([len(p) for p in packets], np.uint32))


def crafted_l7(seed: int = 13) -> list[bytes]:
    """TCP/UDP payloads at the edges of the L7 content checks the engine restates (HTTP request method, HTTP
    response version / status code / status line end, SSL record header, DNS lengths) on HTTP, SSL, DNS and other
    trigger ports, over IPv4 and IPv6, some behind a VLAN tag (generic walk) and padded past the LDS window."""
    rng = np.random.default_rng(seed)
    bodies = [b"GET / HTTP/1.1\r\n", b"GET", b"GET ", b" GET /", b"GETX / HTTP/1.1", b"OPTIONS * HTTP/1.1\r\n",
              b"CONNECT a:443 HTTP/1.1", b"PATCH /x", b"DELETE", b"TRACE / HTTP/1.0\r\n", b"get / HTTP/1.1",
              b"HTTP/1.1 200 OK\r\n", b"HTTP/1.1 200 \r\n", b"HTTP/1.1 200\r\n", b"HTTP/1.1 200 X", b"HTTP/1.0 999 X\n",
              b"HTTP/0.9 404 Not Found\n", b"HTTP/2.0 200 OK\r\n", b"HTTP/1.1 20A OK\r\n", b"HTTP/1.1 599 \r\r\n",
              b"HTTP/1.1 226 IM Used" + b"x" * 150 + b"\n", b"HTTP/1.1 103 E\n",
              bytes([22, 3, 1, 0, 5]) + b"hello", bytes([23, 3, 3, 0, 0]), bytes([24, 3, 3, 1, 0]),
              bytes([20, 0x7f, 0x1c, 0, 1, 1]), bytes([21, 0xfb, 0x1a, 0, 2]), bytes([22, 3, 5, 0, 9]),
              bytes([22, 3, 0, 1, 0]), bytes([22, 3]), b"", b"x" * 11, b"x" * 12, b"x" * 13, b"x" * 14,
              b"INVITE sip:a SIP/2.0\r\n", rng.bytes(40)]
    # the layers built behind a classified first L7 layer: HTTP header fields (TextBasedProtocol.cpp:87-139,
    # 448-461) and first-line ends, SSL record chains (SSLLayer.cpp:88-106), DNS lengths
    bodies += [b"GET /a HTTP/1.1\r\nHost: x\r\nA: b\r\n\r\nbody", b"GET /a HTTP/1.1\r\nHost: x\r\n\r\n",
               b"GET /a HTTP/1.1\nHost: x\n\nbody", b"GET /a HTTP/1.1\r\nHost: x", b"GET /a HTTP/1.1\r\nHost: x\r\n",
               b"GET /a HTTP/1.1\r\nHo\0st: x", b"GET /a HTTP/1.1\r\n\0Host", b"GET /a HTTP/1.1\r\nHo\0st: x\r\n\r\n",
               b"GET /a HTTP/1.1\r\n\r\n", b"GET /a HTTP/1.1\r\n\n", b"GET /a HTTP/1.1\r\n\rX\r\nA: b\r\n",
               b"GET /a HTT", b"GET /a HTTP/1", b"GET /a HTTP/1.", b"GET /a HTTP/1.1", b"GET /a HTTP/7.7\r\nA: b\r\n\r\nz",
               b"GET /a\r\nA: b HTTP/1.1\r\nC: d\r\n\r\n", b"GET  HTTP/1.0\nX", b"POST /p HTTP/1.0\r\nL: 3\r\n\r\nabc" * 3,
               b"HTTP/1.1 200 OK\r\nServer: s\r\nContent-Length: 4\r\n\r\nbody", b"HTTP/1.1 200 OK\r\nA: b",
               b"HTTP/1.1 200 OK\r\n\r\n", b"HTTP/1.1 200 OK\r\nA:\0b\r\n\r\nq", b"HTTP/1.1 404 Not Found\nA: b\n\nzz",
               b"HTTP/1.1 200 OK\r\n" + b"X-Long: " + b"v" * 300 + b"\r\n\r\n" + b"b" * 100,
               bytes([22, 3, 1, 0, 2, 1, 2, 20, 3, 3, 0, 1, 1, 23, 3, 3, 0, 3, 9, 9, 9]),
               bytes([22, 3, 1, 0, 2, 1, 2, 20, 3, 3, 0, 1, 1, 99, 3, 3, 0, 1, 1]), bytes([22, 3, 1, 0, 2, 1, 2, 23, 3]),
               bytes([22, 3, 1, 0, 2, 1, 2, 23, 3, 3, 0, 0]), bytes([22, 3, 1, 0, 2, 1, 2, 23, 3, 3, 0, 9, 1]),
               bytes([23, 3, 3, 0, 40]) + b"e" * 10, bytes([21, 3, 3, 0, 2, 1, 0]) * 12,
               bytes([23, 3, 4, 0, 1, 7]) * 30, bytes([22, 3, 3, 0, 4, 1, 0, 0, 0, 22, 0x7f, 0x10, 0, 1, 1, 22, 3, 6, 0, 1, 1]),
               b"\x12\x34\x01\x00\x00\x01\x00\x00\x00\x00\x00\x00\x03www\x01a\x00\x00\x01\x00\x01",
               b"\x00\x1d\x12\x34\x01\x00\x00\x01\x00\x00\x00\x00\x00\x00\x03www\x01a\x00\x00\x01\x00\x01",
               # SSH messages (SSHLayer.cpp:18-56,135-170): identification, handshake chains, encrypted fall-backs
               b"SSH-2.0-OpenSSH_8.9\r\n", b"SSH-2.0-x", b"SSH-\n", b"SSH\n", b"SSH-1.99-a\n" + b"z" * 200,
               struct.pack(">IBB", 12, 4, 20) + b"k" * 10, struct.pack(">IBB", 6, 2, 21) + b"ab" + struct.pack(">IBB", 2, 0, 30),
               struct.pack(">IBB", 6, 2, 31) + b"ab" + b"\x99" * 33, struct.pack(">IBB", 60, 4, 20) + b"k" * 10,
               struct.pack(">IBB", 8, 9, 20) + b"k" * 6, struct.pack(">IBB", 8, 2, 50) + b"k" * 6,
               struct.pack(">IBB", 8, 2, 49) + b"k" * 6 + struct.pack(">IBB", 0, 0, 20),
               struct.pack(">IBB", 0xFFFFFFFC, 2, 20) + b"k" * 6, (struct.pack(">IBB", 2, 0, 21)) * 25,
               # MySQL (MySqlLayer.cpp:200-340: the layer is the whole payload whatever its messages)
               b"\x05\x00\x00\x00\x03SELECT 1", b"\x07\x00\x00\x01\x00\x00\x00\x02\x00\x00\x00", b"\x01"]
    tcp_ports = [(40000, 80), (80, 40000), (8080, 8080), (443, 40000), (40000, 993), (80, 443), (53, 40000),
                 (40000, 5353), (22, 80), (443, 179), (5060, 80), (102, 443), (21, 8080), (40000, 40001), (2123, 53),
                 (22, 40000), (40000, 22), (22, 5060), (179, 22), (22, 3306), (3306, 40000), (40000, 3306), (3306, 53),
                 (3306, 2123), (502, 3306), (3306, 3306), (5432, 3306), (3306, 443), (23, 3306)]
    udp_ports = [(40000, 53), (53, 40000), (5355, 5355), (68, 67), (67, 53), (40000, 4789), (2152, 53), (53, 2123),
                 (40000, 5060), (40000, 40001), (123, 53), (40000, 9)]
    pk = []
    for body in bodies:
        for sp, dp in tcp_ports:
            l4 = _tcp(sp, dp, body)
            pk.append(_eth(0x0800) + _ipv4(6, len(l4)) + l4)
            pk.append(_eth(0x8100) + struct.pack(">HH", 7, 0x86DD) + _ipv6(6, len(l4)) + l4)
        for sp, dp in udp_ports:
            l4 = _udp(sp, dp, body)
            pk.append(_eth(0x0800) + _ipv4(17, len(l4)) + l4 + bytes(int(rng.integers(0, 3))))
    return pk


def crafted_http(n: int = 1500, seed: int = 29) -> list[bytes]:
    """HTTP requests and responses whose first lines and header fields end at every offset of the engine's text-walk
    groups (2 / 4 payload dwords per read) and far past the LDS window: random URL lengths (with spaces and near-miss
    "HTTP" strings in them), 0-24 header fields of 0-300 bytes ending in CRLF or LF, a NUL now and then, an end of
    header or none, a body or none; over Eth/IPv4 and VLAN/IPv6, port 80 both ways. The device's HTTP layer lengths
    (TextBasedProtocol.cpp:87-139,448-461; HttpLayer.cpp:166-213) against the restatement and the reference."""
    rng = np.random.default_rng(seed)
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-/._=", dtype=np.uint8)

    def text(k: int) -> bytes:
        return bytes(letters[rng.integers(0, len(letters), k)])

    pk = []
    for i in range(n):
        nl = b"\r\n" if rng.random() < 0.7 else b"\n"
        if rng.random() < 0.6:
            url = bytearray(b"/" + text(int(rng.integers(0, 600))))
            for _ in range(int(rng.integers(0, 3))):  # spaces and near-miss versions inside the URL
                at = int(rng.integers(0, len(url) + 1))
                url[at:at] = [b" ", b" HTTP", b" HTTP/", b" HTT", b"HTTP/"][int(rng.integers(0, 5))]
            ver = [b" HTTP/1.1", b" HTTP/1.0", b" HTTP/1", b" HTTP/", b""][int(rng.choice(5, p=[.6, .2, .08, .06, .06]))]
            first = [b"GET ", b"POST ", b"HEAD ", b"OPTIONS "][int(rng.integers(0, 4))] + bytes(url) + ver
            sp, dp = 40000 + i % 1000, 80
        else:
            first = b"HTTP/1.1 " + [b"200 OK", b"404 Not Found", b"301 " + text(int(rng.integers(1, 80)))][
                int(rng.integers(0, 3))]
            sp, dp = 80, 40000 + i % 1000
        msg = first + nl
        for _ in range(int(rng.integers(0, 25))):
            f = text(int(rng.integers(1, 20))) + b": " + text(int(rng.integers(0, 280)))
            if rng.random() < 0.03:
                at = int(rng.integers(0, len(f)))
                f = f[:at] + b"\0" + f[at:]
            msg += f + (nl if rng.random() < 0.97 else b"\n")
        if rng.random() < 0.8:
            msg += nl  # the end of the header
            if rng.random() < 0.5:
                msg += text(int(rng.integers(1, 300)))
        msg = msg[:1400]
        l4 = _tcp(sp, dp, msg)
        if i % 2:
            pk.append(_eth(0x0800) + _ipv4(6, len(l4)) + l4)
        else:
            pk.append(_eth(0x8100) + struct.pack(">HH", 7, 0x86DD) + _ipv6(6, len(l4)) + l4)
    return pk


def crafted_linklayers(seed: int = 23) -> dict[int, list[bytes]]:
    """First layers of the non-Ethernet link types the engine builds, per link type: Linux SLL (113), SLL2 (276),
    Null/Loopback (0), Cisco HDLC (104) and NFLOG (239, its TLV walk: records before, after and without the payload
    record, empty, short and overlong records) at and around their length rules, every protocol / family encoding they dispatch on
    (NullLoopbackLayer::getFamily's byte-order guesses, Packet++/src/NullLoopbackLayer.cpp:23-43), followed by valid
    and broken IPv4 / IPv6 / VLAN / MPLS / ARP / LLC / PPPoE payloads."""
    rng = np.random.default_rng(seed)
    t4, u6 = _tcp(1234, 80, rng.bytes(20)), _udp(5000, 6000, rng.bytes(12))
    ip4 = _ipv4(6, len(t4)) + t4
    ip6 = _ipv6(17, len(u6)) + u6
    inner = {0x0800: [ip4, ip4[:19], b"\x45" + ip4[1:10]], 0x86DD: [ip6, ip6[:39]], 0x8100: [b"\x00\x01\x08\x00" + ip4, b"\x00\x01"],
             0x88A8: [b"\x00\x02\x86\xdd" + ip6], 0x8847: [b"\x00\x01\x41\x40" + ip4, b"\x00"], 0x0806: [bytes(28), bytes(10)],
             0x8864: [bytes(20)], 0x0004: [b"\x42\x42\x03" + bytes(30), b"\xff\xff\x03", b"\xaa\xaa\x03\x00"],
             0x1234: [rng.bytes(30)], 0x05DC: [rng.bytes(8)]}
    out = {113: [], 276: [], 0: []}
    for et, bodies in inner.items():
        for body in bodies:
            out[113].append(rng.bytes(14) + et.to_bytes(2, "big") + body)
            out[276].append(et.to_bytes(2, "big") + rng.bytes(18) + body)
    for n in range(0, 24):
        out[113].append(rng.bytes(n))
        out[276].append(rng.bytes(n))
        out[0].append(rng.bytes(n))
    fams = [2, 24, 28, 30, 7, 0x0800, 0x86DD, 0x1234, 1500, 1501]
    for fam in fams:
        for enc in (fam.to_bytes(4, "little"), fam.to_bytes(4, "big"), (fam << 16).to_bytes(4, "little"),
                    (fam & 0xFFFF).to_bytes(2, "big") + b"\0\0"):
            for body in (ip4, ip6, ip4[:19], b"", rng.bytes(5)):
                out[0].append(enc + body)
    for w in (0x00020000, 0x00050000, 0x00060000, 0x01000000, 0x00000200, 0x00000600, 0x00000002, 0x0000FF00):
        out[0].append(w.to_bytes(4, "little") + ip4)
    # Cisco HDLC (104, CiscoHdlcLayer.cpp:43-67): address, control, protocol (big-endian), then IPv4 / IPv6 / anything
    out[104] = [rng.bytes(n) for n in range(0, 12)]
    for addr in (0x0F, 0x8F, 0x00):
        for proto, bodies in ((0x0800, [ip4, ip4[:19], b"\x46" + ip4[1:]]), (0x86DD, [ip6, ip6[:39]]),
                              (0x8035, [rng.bytes(20)]), (0x0806, [bytes(28)])):
            for body in bodies + [b""]:
                out[104].append(bytes([addr, 0]) + proto.to_bytes(2, "big") + body)

    # NFLOG (239, NflogLayer.cpp:41-96): family, version, resource id, then TLVs {u16 length, u16 type} in host order,
    # each align<4>(length) long; the payload record (type 9) carries the packet
    def tlv(t: int, value: bytes, length: int | None = None) -> bytes:
        ln = 4 + len(value) if length is None else length
        raw = ln.to_bytes(2, "little") + t.to_bytes(2, "little") + value
        return raw + bytes((-len(raw)) % 4)

    out[239] = [rng.bytes(n) for n in range(0, 12)]
    for fam, body in ((2, ip4), (10, ip6), (2, ip4[:19]), (10, ip6[:39]), (7, rng.bytes(20)), (2, ip4 + b"\0\0\0"),
                      (2, b""), (10, ip4)):
        head = bytes([fam, 0]) + (0x002A).to_bytes(2, "big")
        pre = tlv(1, b"\x08\x00\x01\x00") + tlv(10, b"drop\0")  # NFULA_PACKET_HDR, a padded NFULA_PREFIX
        out[239] += [head + pre + tlv(9, body), head + tlv(9, body), head + pre, head + pre + tlv(9, body) + rng.bytes(6),
                     head + tlv(9, body)[:-3], head + tlv(9, body, 4 + len(body) + 40), head + tlv(9, body, 3),
                     head + tlv(1, b"", 0) + tlv(9, body), head + tlv(8, bytes(8)) + tlv(9, body) + tlv(16, bytes(14))]
    # TLV walks past the gathered header window (the device reads them from HBM): 40 empty records (160 B), or one
    # 200-B prefix, before the payload record; a record list that ends on a torn header
    for fam, body in ((2, ip4), (10, ip6)):
        head = bytes([fam, 0]) + (0x002A).to_bytes(2, "big")
        out[239] += [head + tlv(11, b"") * 40 + tlv(9, body), head + tlv(10, rng.bytes(200)) + tlv(9, body),
                     head + tlv(11, b"") * 30 + b"\x09\x00", head + tlv(11, b"") * 25 + tlv(9, body, 2000)]
    return out
