"""Seeded synthetic packet batches for BASELINE.json's configs.

Packets are generated per header template as 2-D arrays (vectorised numpy), with valid IPv4 and L4
checksums, ports drawn outside the reference's L7 trigger sets (so Packet++ yields GenericPayload,
TcpLayer.cpp:372-491 / UdpLayer.cpp:103-178), then laid back to back in a random interleaving order.

  config 1: 10k Eth/IPv4/UDP, caplen uniform 64..1500, seed 1
  config 2: 1M x 64 B Eth/IPv4/{TCP,UDP} 50/50, seed 2
  config 3: 10M IMIX 64/512/1500 B at 7:4:1, 25% single VLAN, 70% IPv4 / 30% IPv6 (64 B: IPv6/UDP
            without VLAN only), TCP/UDP 50/50, 1% corrupted checksums, seed 3
  config 4: IMIX as config 3 with 5-tuples drawn Zipf(1.1) over a flow table, both directions, seed 4
  config 5: deep encapsulation -- QinQ, 1-3 MPLS labels, GREv0 (C/K/S) over IPv4/IPv6, IPv6 with 1-3
            extension headers -- then TCP/UDP, 64/512/1500 B, seed 5
"""
from __future__ import annotations

import numpy as np

from . import abi
from .pcap import PacketBatch

# ports the reference routes to L7 dissectors (engine contract, oracle tcp_l7_port/udp_l7_port)
TRIGGER_PORTS = np.array(sorted({
    443, 261, 448, 465, 563, 614, 636, 989, 990, 992, 993, 994, 995, 80, 8080, 5060, 5061, 179, 22, 53,
    5353, 5355, 23, 21, 20, 13400, 3496, 30490, 102, 25, 587, 389, 5432, 3306, 2123, 502, 67, 68, 4789, 0,
    7, 9, 1812, 1813, 3799, 2152, 546, 547, 123, 51820}), dtype=np.int64)
SIP_KEYS = [b"INVI", b"ACK ", b"BYE ", b"CANC", b"REGI", b"PRAC", b"OPTI", b"SUBS", b"NOTI", b"PUBL",
            b"INFO", b"REFE", b"MESS", b"UPDA", b"SIP/"]

IMIX_SIZES = (64, 512, 1500)
IMIX_WEIGHTS = (7, 4, 1)


def safe_ports(rng: np.random.Generator, n: int) -> np.ndarray:
    p = rng.integers(1024, 65536, size=n, dtype=np.int64)
    bad = np.isin(p, TRIGGER_PORTS)
    while bad.any():
        p[bad] = rng.integers(1024, 65536, size=int(bad.sum()), dtype=np.int64)
        bad = np.isin(p, TRIGGER_PORTS)
    return p.astype(np.uint16)


def _be16(a: np.ndarray) -> np.ndarray:
    a = a.astype(np.uint32)
    return np.stack([(a >> 8) & 0xFF, a & 0xFF], axis=1).astype(np.uint8)


def _le_word_sum(rows: np.ndarray) -> np.ndarray:
    """Sum of little-endian 16-bit words of each row (odd length zero-padded), as uint64."""
    n, w = rows.shape
    if w % 2:
        rows = np.concatenate([rows, np.zeros((n, 1), np.uint8)], axis=1)
    return rows.view("<u2").sum(axis=1, dtype=np.uint64)


def _fold_checksum(s: np.ndarray) -> np.ndarray:
    """computeChecksum's fold + invert, as the 16-bit value stored big-endian in the header."""
    s = s.astype(np.uint64)
    while (s >> 16).any():
        s = (s & 0xFFFF) + (s >> 16)
    res = (~s) & 0xFFFF  # little-endian word sum, inverted: written back as LE bytes
    return res.astype(np.uint16)


def _be32(a: np.ndarray) -> np.ndarray:
    a = a.astype(np.uint64)
    return np.stack([(a >> 24) & 0xFF, (a >> 16) & 0xFF, (a >> 8) & 0xFF, a & 0xFF], axis=1).astype(np.uint8)


def _ipv4_header(rows: np.ndarray, ip: int, proto: int, total: int) -> None:
    """IPv4 header without options at column ip (addresses and id keep their random bytes); the checksum
    is set by _ipv4_checksum once every header byte is final."""
    n = rows.shape[0]
    rows[:, ip] = 0x45
    rows[:, ip + 1] = 0
    rows[:, ip + 2:ip + 4] = _be16(np.full(n, total))
    rows[:, ip + 6] = 0x40  # DF, offset 0
    rows[:, ip + 7] = 0
    rows[:, ip + 8] = 64
    rows[:, ip + 9] = proto
    rows[:, ip + 10:ip + 12] = 0


def _ipv4_checksum(rows: np.ndarray, ip: int) -> None:
    rows[:, ip + 10:ip + 12] = 0
    c = _fold_checksum(_le_word_sum(rows[:, ip:ip + 20]))
    rows[:, ip + 10] = (c & 0xFF).astype(np.uint8)
    rows[:, ip + 11] = (c >> 8).astype(np.uint8)


def _ipv6_header(rows: np.ndarray, ip: int, next_header: int, payload_len: int) -> None:
    n = rows.shape[0]
    rows[:, ip] = 0x60 | (rows[:, ip] & 0x0F)
    rows[:, ip + 4:ip + 6] = _be16(np.full(n, payload_len))
    rows[:, ip + 6] = next_header
    rows[:, ip + 7] = 64


def _put_l4(rows: np.ndarray, ip: int, ipv6: bool, l4o: int, tcp: bool, sport: np.ndarray,
            dport: np.ndarray) -> None:
    """TCP (20 B) or UDP header at l4o with a valid checksum over the rest of the row, the pseudo header
    taken from the IP header at ip (computePseudoHdrChecksum, PacketUtils.cpp:66-112)."""
    n, size = rows.shape
    l4len = size - l4o
    proto = 6 if tcp else 17
    rows[:, l4o:l4o + 2] = _be16(sport)
    rows[:, l4o + 2:l4o + 4] = _be16(dport)
    if tcp:
        rows[:, l4o + 12] = 0x50
        rows[:, l4o + 13] = 0x18
        rows[:, l4o + 16:l4o + 20] = 0
        cs = l4o + 16
    else:
        rows[:, l4o + 4:l4o + 6] = _be16(np.full(n, l4len))
        rows[:, l4o + 6:l4o + 8] = 0
        cs = l4o + 6
        # keep the UDP payload clear of the SIP content heuristic (SipLayer.cpp:127-160)
        if l4len - 8 >= 4:
            head = rows[:, l4o + 8:l4o + 12].copy().view(">u4").ravel()
            keys = np.array([int.from_bytes(k, "big") for k in SIP_KEYS], dtype=np.uint32)
            hit = np.isin(head, keys)
            rows[hit, l4o + 8] ^= 0x80
    s = _le_word_sum(rows[:, l4o:])
    addr_lo, addr_hi = (ip + 8, ip + 40) if ipv6 else (ip + 12, ip + 20)
    s += _le_word_sum(rows[:, addr_lo:addr_hi])
    s += np.uint64(((l4len & 0xFF) << 8) | (l4len >> 8))
    s += np.uint64(proto << 8)
    c = _fold_checksum(s)
    if not tcp:
        c = np.where(c == 0, np.uint16(0xFFFF), c)
    rows[:, cs] = (c & 0xFF).astype(np.uint8)
    rows[:, cs + 1] = (c >> 8).astype(np.uint8)


def build_rows(rng: np.random.Generator, n: int, size: int, vlan: bool, ipv6: bool, tcp: bool,
               tuples: dict | None = None) -> np.ndarray:
    """n packets of `size` bytes: Eth [VLAN] IPv4|IPv6 TCP|UDP + random payload, valid checksums."""
    l2 = 18 if vlan else 14
    l3 = 40 if ipv6 else 20
    l4 = 20 if tcp else 8
    hlen = l2 + l3 + l4
    if hlen > size:
        raise ValueError("headers do not fit")
    rows = np.frombuffer(rng.bytes(n * size), dtype=np.uint8).reshape(n, size).copy()
    # Ethernet (EthLayer.h ether_header): dst, src, ethertype
    et = 0x86DD if ipv6 else 0x0800
    if vlan:
        rows[:, 12:14] = _be16(np.full(n, 0x8100))
        tci = rng.integers(1, 4095, size=n)
        rows[:, 14:16] = _be16(tci)
        rows[:, 16:18] = _be16(np.full(n, et))
    else:
        rows[:, 12:14] = _be16(np.full(n, et))
    rows[:, 0] &= 0xFE  # unicast dst
    ip = l2
    l4o = l2 + l3
    if tuples is not None:
        src_ip, dst_ip, sport, dport = tuples["src"], tuples["dst"], tuples["sport"], tuples["dport"]
    else:
        src_ip = dst_ip = None
        sport, dport = safe_ports(rng, n), safe_ports(rng, n)
    proto = 6 if tcp else 17
    if ipv6:
        _ipv6_header(rows, ip, proto, size - l4o)
        if src_ip is not None:
            rows[:, ip + 8:ip + 24] = src_ip
            rows[:, ip + 24:ip + 40] = dst_ip
    else:
        _ipv4_header(rows, ip, proto, size - l2)
        if src_ip is not None:
            rows[:, ip + 12:ip + 16] = src_ip
            rows[:, ip + 16:ip + 20] = dst_ip
        _ipv4_checksum(rows, ip)
    _put_l4(rows, ip, ipv6, l4o, tcp, sport, dport)
    return rows


# ---- config 5: deep encapsulation ----
K5_PLAIN, K5_MPLS, K5_GRE, K5_EXT = 0, 1, 2, 3
# IPv6 extension chains: (extension ids, Hdr Ext Len byte of each); 0 Hop-by-Hop, 60 Destination,
# 43 Routing use 8*(len+1) bytes, 44 Fragment 8 (IPv6Extensions.h:40-43); a last Fragment header makes the
# rest a Payload (IPv6Layer.cpp:194-312)
DEEP_EXT = (((0,), (0,)), ((60,), (1,)), ((43,), (2,)), ((0, 60), (0, 1)), ((0, 43), (1, 0)),
            ((43, 60), (0, 0)), ((0, 43, 60), (0, 1, 0)), ((0, 44), (0, 0)), ((60, 44), (2, 0)),
            ((0, 60, 44), (0, 0, 0)))
# template variants per kind: plain 1; MPLS 1-3 labels; GRE outer IPv4/IPv6 (bit 3) x C/K/S option bits
# (bits 0-2); IPv6 extension chain index
DEEP_VARIANTS = (1, 3, 16, len(DEEP_EXT))


def _deep_hlen(l2: int, kind: int, var: int, inner_v6: bool, tcp: bool) -> int:
    h = 14 + 4 * l2
    if kind == K5_MPLS:
        h += 4 * (var + 1)
    elif kind == K5_GRE:
        h += (40 if var >> 3 else 20) + 4 + 4 * bin(var & 7).count("1")
    if kind == K5_EXT:
        chain, hls = DEEP_EXT[var]
        h += 40 + sum(8 if t == 44 else 8 * (hl + 1) for t, hl in zip(chain, hls))
    else:
        h += 40 if inner_v6 else 20
    return h + (20 if tcp else 8)


def build_deep_rows(rng: np.random.Generator, n: int, size: int, l2: int, kind: int, var: int, inner_v6: bool,
                    tcp: bool) -> np.ndarray:
    """n packets of `size` bytes with one config-5 stack: Ethernet, then none / one 802.1Q tag / QinQ
    (0x88A8 + 0x8100), then plain IP, an MPLS label stack (1-3), IPv4|IPv6 + GREv0 with C/K/S options, or
    IPv6 with extension headers, then TCP|UDP + random payload. Valid IPv4 header and L4 checksums."""
    rows = np.frombuffer(rng.bytes(n * size), dtype=np.uint8).reshape(n, size).copy()
    rows[:, 0] &= 0xFE
    v6 = inner_v6 or kind == K5_EXT
    inner_et = 0x86DD if v6 else 0x0800
    if kind == K5_MPLS:
        et = 0x8847
    elif kind == K5_GRE:
        et = 0x86DD if var >> 3 else 0x0800
    else:
        et = inner_et
    tags = (0x88A8, 0x8100)[2 - l2:] if l2 else ()
    seq = (*tags, et)
    rows[:, 12:14] = _be16(np.full(n, seq[0]))
    pos = 14
    for t in range(len(tags)):
        rows[:, pos:pos + 2] = _be16(rng.integers(1, 4095, size=n))
        rows[:, pos + 2:pos + 4] = _be16(np.full(n, seq[t + 1]))
        pos += 4
    v4 = []
    if kind == K5_MPLS:  # label(20) TC(3) S(1) TTL(8); S is bit 0 of byte 2 (MplsLayer.cpp:25-28)
        for k in range(var + 1):
            label = rng.integers(16, 1 << 20, size=n, dtype=np.int64)
            rows[:, pos:pos + 4] = _be32((label << 12) | ((1 if k == var else 0) << 8) | 64)
            pos += 4
    elif kind == K5_GRE:  # GREv0: C 0x80, K 0x20, S 0x10 of byte 0 (GreLayer.h:14-57)
        if var >> 3:
            _ipv6_header(rows, pos, 47, size - pos - 40)
            pos += 40
        else:
            _ipv4_header(rows, pos, 47, size - pos)
            v4.append(pos)
            pos += 20
        flags = var & 7
        rows[:, pos] = (0x80 if flags & 1 else 0) | (0x20 if flags & 2 else 0) | (0x10 if flags & 4 else 0)
        rows[:, pos + 1] = 0
        rows[:, pos + 2:pos + 4] = _be16(np.full(n, inner_et))
        pos += 4 + 4 * bin(flags).count("1")
    ip = pos
    proto = 6 if tcp else 17
    if kind == K5_EXT:
        chain, hls = DEEP_EXT[var]
        _ipv6_header(rows, ip, chain[0], size - ip - 40)
        e = ip + 40
        for t, nh, hl in zip(chain, (*chain[1:], proto), hls):
            rows[:, e] = nh
            rows[:, e + 1] = 0 if t == 44 else hl
            e += 8 if t == 44 else 8 * (hl + 1)
        l4o = e
    elif v6:
        _ipv6_header(rows, ip, proto, size - ip - 40)
        l4o = ip + 40
    else:
        _ipv4_header(rows, ip, proto, size - ip)
        v4.append(ip)
        l4o = ip + 20
    _put_l4(rows, ip, v6, l4o, tcp, safe_ports(rng, n), safe_ports(rng, n))
    for h in v4:
        _ipv4_checksum(rows, h)
    return rows


def _deep_decode(c: int) -> tuple[int, int, int, bool, bool]:
    tcp, c = c & 1, c >> 1
    v6, c = c & 1, c >> 1
    var, c = c % 16, c // 16
    return int(c // 4), int(c % 4), int(var), bool(v6), bool(tcp)


def deep(n: int, seed: int = 5, sizes=IMIX_SIZES, weights=IMIX_WEIGHTS) -> PacketBatch:
    """Config 5: deep-encapsulation stress. Sizes 64/512/1500 B at 7:4:1 where the stack fits (else
    512 B); stacks (build_deep_rows): plain IP 10%, MPLS 30%, GRE 30%, IPv6 extensions 30%; no tag 30%,
    one VLAN tag 20%, QinQ 50%; inner IPv4/IPv6 50/50; TCP/UDP 50/50."""
    rng = np.random.default_rng(seed)
    w = np.array(weights, dtype=np.float64)
    size_idx = rng.choice(len(sizes), size=n, p=w / w.sum())
    l2 = rng.choice(3, size=n, p=[0.3, 0.2, 0.5])
    kind = rng.choice(4, size=n, p=[0.1, 0.3, 0.3, 0.3])
    var = rng.integers(0, 1 << 30, size=n) % np.array(DEEP_VARIANTS)[kind]
    inner_v6 = (rng.random(n) < 0.5) | (kind == K5_EXT)
    tcp = rng.random(n) < 0.5
    code = ((((l2 * 4 + kind) * 16 + var) * 2 + inner_v6) * 2 + tcp).astype(np.int64)
    codes, inv = np.unique(code, return_inverse=True)
    hlen = np.array([_deep_hlen(*_deep_decode(int(c))) for c in codes])[inv]
    size_idx = np.where(np.array(sizes)[size_idx] < hlen, 1, size_idx)
    key = code * len(sizes) + size_idx
    order = np.argsort(key, kind="stable")
    ukeys, starts = np.unique(key[order], return_index=True)
    bounds = np.append(starts, n)
    groups = []
    for g, k in enumerate(ukeys):
        c, si = divmod(int(k), len(sizes))
        idx = order[bounds[g]:bounds[g + 1]]
        grng = np.random.default_rng([seed, c, si])
        groups.append((build_deep_rows(grng, len(idx), sizes[si], *_deep_decode(c)), idx))
    batch = _interleave(groups, n, rng)
    del groups
    batch.meta.update(config="deep", seed=seed)
    return batch


def _interleave(groups: list[tuple[np.ndarray, np.ndarray]], n: int, order_rng: np.random.Generator,
                chunk_bytes: int = 1 << 26) -> PacketBatch:
    """groups: (rows[n_g, size_g], packet indices[n_g]) -> back-to-back batch in index order."""
    caps = np.zeros(n, dtype=np.uint32)
    for rows, idx in groups:
        caps[idx] = rows.shape[1]
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        np.cumsum(caps[:-1], dtype=np.uint64, out=offs[1:])
    total = int(offs[-1]) + int(caps[-1]) if n else 0
    data = np.empty(total + 64, dtype=np.uint8)
    data[total:] = 0
    for rows, idx in groups:
        size = rows.shape[1]
        step = max(1, chunk_bytes // size)
        col = np.arange(size, dtype=np.int64)
        for a in range(0, len(idx), step):
            d = offs[idx[a:a + step]].astype(np.int64)
            data[(d[:, None] + col[None, :]).ravel()] = rows[a:a + step].ravel()
    return PacketBatch(data, offs, caps, abi.LINKTYPE_ETHERNET)


def _corrupt(batch: PacketBatch, rng: np.random.Generator, frac: float, info: dict) -> None:
    """Flip checksum bytes of a fraction of packets (config 3's 1% corrupted checksums)."""
    n = batch.n
    k = int(n * frac)
    if k == 0:
        return
    pick = rng.choice(n, size=k, replace=False)
    half = pick[: k // 2]
    rest = pick[k // 2:]
    l4cs = info["l4_csum_off"]
    ipcs = info["ip_csum_off"]
    offs = batch.offsets.astype(np.int64)
    batch.data[offs[half] + l4cs[half]] ^= 0x5A
    v4 = rest[ipcs[rest] > 0]
    batch.data[offs[v4] + ipcs[v4]] ^= 0xA5
    batch.meta["corrupted"] = int(len(half) + len(v4))


def _imix_attrs(rng: np.random.Generator, n: int, vlan_frac: float, v6_frac: float, sizes, weights,
                flows: int | None, univ: dict | None) -> dict:
    """Per-packet draws of an IMIX batch: size, VLAN, IPv6, TCP, and with a flow universe the Zipf(1.1) flow and the
    direction (the flow then fixes IPv6 / TCP)."""
    w = np.array(weights, dtype=np.float64)
    size_of = np.array(sizes)[rng.choice(len(sizes), size=n, p=w / w.sum())]
    vlan = rng.random(n) < vlan_frac
    v6 = rng.random(n) < v6_frac
    tcp = rng.random(n) < 0.5
    small = size_of < 14 + 4 + 40 + 20 + 2
    # 64 B: IPv6 only as IPv6/UDP without VLAN (14+40+8 = 62 fits; 66/82 do not)
    tcp = np.where(small & v6, False, tcp)
    vlan = np.where(small & v6, False, vlan)
    flow_id = dirn = None
    if flows:
        ranks = np.arange(1, flows + 1, dtype=np.float64)
        pz = ranks ** -1.1
        pz /= pz.sum()
        flow_id = rng.choice(flows, size=n, p=pz)
        dirn = rng.random(n) < 0.5
        v6 = univ["v6"][flow_id]
        tcp = univ["tcp"][flow_id]
        # a flow keeps its protocol: 64 B cannot hold IPv6/TCP, so those packets become 512 B
        size_of = np.where(small & v6 & tcp, sizes[1], size_of)
        small = size_of < 14 + 4 + 40 + 20 + 2
        vlan = np.where(small & v6, False, vlan)
    return {"size_of": size_of, "vlan": vlan, "v6": v6, "tcp": tcp, "flow_id": flow_id, "dirn": dirn}


def _flow_universe(seed: int, flows: int, v6_frac: float) -> dict:
    """The flows' 5-tuples (protocol, addresses, ports), drawn from the config's seed alone."""
    frng = np.random.default_rng(seed + 1000)
    u = {"v6": frng.random(flows) < v6_frac, "tcp": frng.random(flows) < 0.5}
    u["src4"] = frng.integers(0, 256, size=(flows, 4), dtype=np.uint8)
    u["dst4"] = frng.integers(0, 256, size=(flows, 4), dtype=np.uint8)
    u["src6"] = frng.integers(0, 256, size=(flows, 16), dtype=np.uint8)
    u["dst6"] = frng.integers(0, 256, size=(flows, 16), dtype=np.uint8)
    u["sp"], u["dp"] = safe_ports(frng, flows), safe_ports(frng, flows)
    return u


def _imix_rows(at: dict, univ: dict | None, n: int, row_seed, sizes, rng: np.random.Generator,
               corrupt_frac: float) -> PacketBatch:
    """Build and interleave the packets the attribute draws describe (groups of one size / VLAN / IP / L4 shape)."""
    size_of, vlan, v6, tcp, flow_id, dirn = (at[k] for k in ("size_of", "vlan", "v6", "tcp", "flow_id", "dirn"))
    groups = []
    info_l4 = np.zeros(n, dtype=np.int64)
    info_ip = np.zeros(n, dtype=np.int64)
    for s in sizes:
        for vl in (False, True):
            for ip6 in (False, True):
                for t in (False, True):
                    idx = np.nonzero((size_of == s) & (vlan == vl) & (v6 == ip6) & (tcp == t))[0]
                    if len(idx) == 0:
                        continue
                    tuples = None
                    if univ is not None:
                        fid = flow_id[idx]
                        fwd = ~dirn[idx]
                        if ip6:
                            a, b = univ["src6"][fid], univ["dst6"][fid]
                        else:
                            a, b = univ["src4"][fid], univ["dst4"][fid]
                        src = np.where(fwd[:, None], a, b)
                        dst = np.where(fwd[:, None], b, a)
                        sp = np.where(fwd, univ["sp"][fid], univ["dp"][fid]).astype(np.uint16)
                        dp = np.where(fwd, univ["dp"][fid], univ["sp"][fid]).astype(np.uint16)
                        tuples = {"src": src, "dst": dst, "sport": sp, "dport": dp}
                    grng = np.random.default_rng([*row_seed, s, int(vl), int(ip6), int(t)])
                    rows = build_rows(grng, len(idx), s, vl, ip6, t, tuples)
                    groups.append((rows, idx))
                    l2 = 18 if vl else 14
                    l4o = l2 + (40 if ip6 else 20)
                    info_l4[idx] = l4o + (16 if t else 6)
                    info_ip[idx] = 0 if ip6 else l2 + 10
    batch = _interleave(groups, n, rng)
    del groups
    if corrupt_frac:
        _corrupt(batch, rng, corrupt_frac, {"l4_csum_off": info_l4, "ip_csum_off": info_ip})
    return batch


def imix(n: int, seed: int, vlan_frac: float = 0.25, v6_frac: float = 0.30, corrupt_frac: float = 0.01,
         sizes=IMIX_SIZES, weights=IMIX_WEIGHTS, flows: int | None = None) -> PacketBatch:
    """Config 3 (flows=None) / an IMIX batch with 5-tuples Zipf(1.1) over `flows` flows, both directions."""
    rng = np.random.default_rng(seed)
    univ = _flow_universe(seed, flows, v6_frac) if flows else None
    at = _imix_attrs(rng, n, vlan_frac, v6_frac, sizes, weights, flows, univ)
    batch = _imix_rows(at, univ, n, [seed], sizes, rng, corrupt_frac)
    batch.meta.update(config="imix", seed=seed, flows=flows)
    if flows:
        batch.meta["flow_id"] = at["flow_id"]
    return batch


FLOW_STREAM_BLOCK = 500_000  # packets per independently drawn block of the config-4 stream


def flow_stream(lo: int, hi: int, seed: int = 4, flows: int = 1_000_000, v6_frac: float = 0.30,
                sizes=IMIX_SIZES, weights=IMIX_WEIGHTS) -> PacketBatch:
    """Packets [lo, hi) of BASELINE config 4's ONE IMIX stream (100M packets over one universe
    of 1M flows, Zipf(1.1) 5-tuples in both directions, cut into contiguous shards, §8e). The stream is drawn in blocks
    of FLOW_STREAM_BLOCK packets, block b from its own seed (seed, b), so any range is generated without the packets
    before it; the flow universe comes from the config's seed alone, so every rank's shard draws from the same 1M
    flows and a flow spans shards. A packet's size, direction and flow -- hence its caplen and hash5Tuple key -- are
    those of the stream position, whichever rank generates it."""
    if not 0 <= lo <= hi:
        raise ValueError("bad stream range")
    n = hi - lo
    univ = _flow_universe(seed, flows, v6_frac)
    parts = []
    for blk in range(lo // FLOW_STREAM_BLOCK, -(-hi // FLOW_STREAM_BLOCK) if n else lo // FLOW_STREAM_BLOCK):
        b0 = blk * FLOW_STREAM_BLOCK
        at = _imix_attrs(np.random.default_rng([seed, 7, blk]), FLOW_STREAM_BLOCK, 0.25, v6_frac, sizes, weights, flows,
                         univ)
        a, e = max(lo, b0) - b0, min(hi, b0 + FLOW_STREAM_BLOCK) - b0
        parts.append({k: v[a:e] for k, v in at.items()})
    at = {k: np.concatenate([p[k] for p in parts]) if parts else np.zeros(0) for k in parts[0]} if parts else \
        _imix_attrs(np.random.default_rng([seed, 7]), 0, 0.25, v6_frac, sizes, weights, flows, univ)
    batch = _imix_rows(at, univ, n, [seed, 7, lo], sizes, np.random.default_rng([seed, 8, lo]), 0.0)
    batch.meta.update(config="flow-stream", seed=seed, flows=flows, stream_lo=lo, stream_hi=hi,
                      flow_id=at["flow_id"])
    return batch


def small64(n: int, seed: int = 2) -> PacketBatch:
    """Config 2: n x 64 B Eth/IPv4/{TCP,UDP} 50/50, valid checksums."""
    rng = np.random.default_rng(seed)
    tcp = rng.random(n) < 0.5
    groups = []
    for t in (False, True):
        idx = np.nonzero(tcp == t)[0]
        if len(idx):
            groups.append((build_rows(np.random.default_rng([seed, int(t)]), len(idx), 64, False, False, t), idx))
    b = _interleave(groups, n, rng)
    b.meta.update(config="64B", seed=seed)
    return b


def udp_uniform(n: int, seed: int = 1, lo: int = 64, hi: int = 1500) -> PacketBatch:
    """Config 1: Eth/IPv4/UDP with caplen uniform in [lo, hi]."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(lo, hi + 1, size=n)
    groups = []
    for s in np.unique(sizes):
        idx = np.nonzero(sizes == s)[0]
        groups.append((build_rows(np.random.default_rng([seed, int(s)]), len(idx), int(s), False, False, False), idx))
    b = _interleave(groups, n, rng)
    b.meta.update(config="udp-uniform", seed=seed)
    return b


def config(cfg: int, n: int | None = None) -> PacketBatch:
    if cfg == 1:
        return udp_uniform(n or 10_000, 1)
    if cfg == 2:
        return small64(n or 1_000_000, 2)
    if cfg == 3:
        return imix(n or 10_000_000, 3)
    if cfg == 4:  # the first n packets of the one config-4 stream (rank 0's shard)
        return flow_stream(0, n or 12_500_000, 4)
    if cfg == 5:
        return deep(n or 10_000_000, 5)
    raise ValueError(f"unknown config {cfg}")
