"""TEST INFRASTRUCTURE ONLY — the parity checkers for the HIP engine.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package. It
loads two C libraries built by oracle/Makefile:
  liboracle.so          — our plain-C restatement of the Packet++ parse path (pcppx_oracle.c)
  _ref/libpcpp_ref.so   — the real reference Packet++ compiled from /root/reference sources, plus our
                          harness (ref_harness.cpp); present only where it was built.
Neither is ever used by the product path (pcapplusplus_amd/), which fails loudly without its HIP library.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from pcapplusplus_amd import abi

ORACLE_DIR = Path(__file__).resolve().parent
ORACLE_SO = ORACLE_DIR / "liboracle.so"
REF_SO = ORACLE_DIR / "_ref" / "libpcpp_ref.so"

_oracle = None
_ref = None


def oracle_lib() -> C.CDLL:
    global _oracle
    if _oracle is None:
        if not ORACLE_SO.exists():
            raise RuntimeError(f"{ORACLE_SO} missing: run `make -C oracle oracle`")
        lib = C.CDLL(str(ORACLE_SO))
        lib.pcppx_oracle_parse_batch.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.Opts),
                                                 C.POINTER(abi.Records), C.c_int]
        lib.pcppx_oracle_parse_batch.restype = C.c_int
        lib.pcppx_oracle_bench.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.Opts), C.c_int,
                                           C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
        lib.pcppx_oracle_bench.restype = C.c_int
        lib.pcppx_oracle_checksum.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_uint32), C.c_int]
        lib.pcppx_oracle_checksum.restype = C.c_uint16
        lib.pcppx_oracle_fnv1.argtypes = [C.c_void_p, C.c_uint32]
        lib.pcppx_oracle_fnv1.restype = C.c_uint32
        lib.pcppx_oracle_reasm_batch.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.Records), C.c_uint8, C.c_void_p]
        lib.pcppx_oracle_reasm_batch.restype = C.c_int
        _oracle = lib
    return _oracle


def ref_available() -> bool:
    return REF_SO.exists()


def ref_lib() -> C.CDLL:
    global _ref
    if _ref is None:
        if not REF_SO.exists():
            raise RuntimeError(f"{REF_SO} missing: build it with `make -C oracle ref` where /root/reference exists")
        lib = C.CDLL(str(REF_SO))
        lib.pcppx_ref_parse_batch.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.Opts), C.POINTER(abi.Records)]
        lib.pcppx_ref_parse_batch.restype = C.c_int
        lib.pcppx_ref_bench.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.Opts), C.c_int,
                                        C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
        lib.pcppx_ref_bench.restype = C.c_int
        lib.pcppx_ref_filter.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.MatchSpec), C.c_void_p,
                                         C.POINTER(abi.PacketStats)]
        lib.pcppx_ref_filter.restype = C.c_int
        lib.pcppx_ref_reasm.argtypes = [C.POINTER(abi.Batch), C.c_void_p]
        lib.pcppx_ref_reasm.restype = C.c_int
        lib.pcppx_ref_tuples.argtypes = [C.POINTER(abi.Batch), C.c_void_p]
        lib.pcppx_ref_tuples.restype = C.c_int
        lib.ref_read_capture.argtypes = [C.c_char_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
        lib.ref_read_capture.restype = C.c_int
        _ref = lib
    return _ref


def _alloc(n: int, opts: abi.Opts):
    summary = np.zeros(n, dtype=abi.SUMMARY_DTYPE)
    layers = np.zeros(max(n * opts.max_layers, 1), dtype=abi.LAYER_DTYPE)
    rec = abi.Records(summary.ctypes.data, layers.ctypes.data if opts.max_layers else None)
    return summary, layers, rec


def oracle_parse(batch, opts: abi.Opts | None = None, threads: int = 1):
    """Restatement records for a PacketBatch: (summary[n], layers[n, max_layers])."""
    opts = opts or abi.make_opts()
    summary, layers, rec = _alloc(batch.n, opts)
    b = batch.c_batch()
    rc = oracle_lib().pcppx_oracle_parse_batch(C.byref(b), C.byref(opts), C.byref(rec), threads)
    if rc != 0:
        raise RuntimeError(f"oracle parse failed {rc}")
    return summary, layers[: batch.n * opts.max_layers].reshape(batch.n, opts.max_layers)


def oracle_parse_tuples(batch, opts: abi.Opts | None = None, threads: int = 1):
    """Restatement records plus the 5-tuple extracts: (summary[n], layers[n, max_layers], tuples[n])."""
    opts = opts or abi.make_opts()
    summary, layers, rec = _alloc(batch.n, opts)
    tuples = np.zeros(max(batch.n, 1), dtype=abi.TUPLE_DTYPE)
    rec.tuples = tuples.ctypes.data
    b = batch.c_batch()
    rc = oracle_lib().pcppx_oracle_parse_batch(C.byref(b), C.byref(opts), C.byref(rec), threads)
    if rc != 0:
        raise RuntimeError(f"oracle parse failed {rc}")
    return summary, layers[: batch.n * opts.max_layers].reshape(batch.n, opts.max_layers), tuples[: batch.n]


def ref_tuples(batch):
    """The 5-tuple extract through the real reference's accessors (oracle/ref_harness.cpp pcppx_ref_tuples) under
    Packet(&raw): tuples[n] with flags 0 and the uncapped chain length in n_layers."""
    out = np.zeros(max(batch.n, 1), dtype=abi.TUPLE_DTYPE)
    b = batch.c_batch()
    rc = ref_lib().pcppx_ref_tuples(C.byref(b), out.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"reference tuples failed {rc}")
    return out[: batch.n]


def proto_stats(summary) -> dict:
    """collectStats totals (PacketStats::collectStats, Common.h:83-104) of engine-format summaries, as the device's
    pcppx_records.proto_stats counts them: the protocol counters from proto_mask for every packet; HTTP / DNS / SSL
    over the settled packets (stats_settled); needs_host = the others."""
    settled, l7 = stats_settled(None, summary, None)
    m = summary["proto_mask"].astype(np.uint64)
    bit = lambda p: int((((m >> np.uint64(p)) & np.uint64(1)) != 0).sum())  # noqa: E731
    return {"packet_count": len(summary), "eth_count": bit(P_ETH), "arp_count": bit(P_ARP), "ipv4_count": bit(P_IPV4),
            "ipv6_count": bit(P_IPV6), "tcp_count": bit(P_TCP), "udp_count": bit(P_UDP),
            "http_count": int((settled & ((l7 & 1) != 0)).sum()), "dns_count": int((settled & ((l7 & 2) != 0)).sum()),
            "tls_count": int((settled & ((l7 & 4) != 0)).sum()), "needs_host_count": int((~settled).sum())}


def compare_tuples(eng, ref, eng_summary=None) -> dict:
    """Engine 5-tuple extracts against the reference's (ref_tuples): every field of every unflagged packet (flags
    aside; n_layers where the chain fits 16 layers). Flagged packets (PCPPX_F_NEEDS_HOST) are the host's."""
    fl = eng["flags"] if eng_summary is None else eng_summary["flags"]
    ok = (fl & abi.F_NEEDS_HOST) == 0
    for f in ("src_ip", "dst_ip", "src_port", "dst_port", "ip_version", "ip_proto", "l4_proto", "has_5tuple", "hash5"):
        a, b = eng[f], ref[f]
        diff = (a != b).reshape(len(a), -1).any(axis=1)
        bad = np.nonzero(ok & diff)[0]
        if len(bad):
            i = int(bad[0])
            raise AssertionError(f"tuple.{f} differs on {len(bad)} unflagged packets; first #{i}: {eng[i]} vs {ref[i]}")
    deep = ref["n_layers"] <= abi.MAX_LAYERS
    bad = np.nonzero(ok & deep & (eng["n_layers"] != ref["n_layers"]))[0]
    if len(bad):
        i = int(bad[0])
        raise AssertionError(f"tuple.n_layers differs on {len(bad)} packets; first #{i}: {eng[i]} vs {ref[i]}")
    return {"n": len(eng), "exact": int(ok.sum()), "with_5tuple": int((ok & (eng["has_5tuple"] != 0)).sum())}


def ref_read_capture(path) -> dict | None:
    """Every packet of a capture as the reference's own file device reads it (PcapFileReaderDevice /
    PcapNgFileReaderDevice getNextPacket, oracle/ref_ingest.cpp): None if the device does not open, else
    {data, caplens, frame_lens, ts_ns, linktypes} (numpy arrays; data back to back)."""
    lib = ref_lib()
    size = max(Path(path).stat().st_size, 1)
    cap_bytes, cap_n = 2 * size + 4096, size // 8 + 64
    while True:
        data = np.empty(cap_bytes, np.uint8)
        cl, fl, lt = (np.empty(cap_n, np.uint32) for _ in range(3))
        ts = np.empty(cap_n, np.uint64)
        used = C.c_uint64(0)
        n = lib.ref_read_capture(str(path).encode(), data.ctypes.data, cap_bytes, cl.ctypes.data, fl.ctypes.data,
                                 ts.ctypes.data, lt.ctypes.data, cap_n, C.byref(used))
        if n == -1:
            return None
        if n == -2:
            cap_bytes, cap_n = cap_bytes * 4, cap_n * 4
            continue
        return {"data": data[: used.value].copy(), "caplens": cl[:n].copy(), "frame_lens": fl[:n].copy(),
                "ts_ns": ts[:n].copy(), "linktypes": lt[:n].copy()}


def ref_parse(batch, opts: abi.Opts | None = None):
    """Real reference Packet++ records for a PacketBatch."""
    opts = opts or abi.make_opts()
    summary, layers, rec = _alloc(batch.n, opts)
    b = batch.c_batch()
    rc = ref_lib().pcppx_ref_parse_batch(C.byref(b), C.byref(opts), C.byref(rec))
    if rc != 0:
        raise RuntimeError(f"reference parse failed {rc}")
    return summary, layers[: batch.n * opts.max_layers].reshape(batch.n, opts.max_layers)


def oracle_bench(batch, opts: abi.Opts, threads: int) -> tuple[float, int]:
    sec, dig = C.c_double(0), C.c_uint64(0)
    b = batch.c_batch()
    rc = oracle_lib().pcppx_oracle_bench(C.byref(b), C.byref(opts), threads, C.byref(sec), C.byref(dig))
    if rc != 0:
        raise RuntimeError("oracle bench failed")
    return sec.value, dig.value


def ref_bench(batch, opts: abi.Opts, threads: int) -> tuple[float, int]:
    sec, dig = C.c_double(0), C.c_uint64(0)
    b = batch.c_batch()
    rc = ref_lib().pcppx_ref_bench(C.byref(b), C.byref(opts), threads, C.byref(sec), C.byref(dig))
    if rc != 0:
        raise RuntimeError("reference bench failed")
    return sec.value, dig.value


def make_spec(src_ip: str | int = 0, dst_ip: str | int = 0, src_port: int = 0, dst_port: int = 0,
              protocol: int = 0) -> abi.MatchSpec:
    sip = abi.ipv4_to_int(src_ip) if isinstance(src_ip, str) else int(src_ip)
    dip = abi.ipv4_to_int(dst_ip) if isinstance(dst_ip, str) else int(dst_ip)
    return abi.MatchSpec(sip, dip, src_port, dst_port, protocol)


def ref_filter(batch, spec: abi.MatchSpec):
    """The reference FilterTraffic worker loop (real PacketMatchingEngine + hash5Tuple flow table +
    collectStats) over a host batch: (matched u8[n], stats dict)."""
    matched = np.zeros(max(batch.n, 1), dtype=np.uint8)
    st = abi.PacketStats()
    b = batch.c_batch()
    rc = ref_lib().pcppx_ref_filter(C.byref(b), C.byref(spec), matched.ctypes.data, C.byref(st))
    if rc != 0:
        raise RuntimeError(f"reference filter failed {rc}")
    return matched[: batch.n], st.as_dict()


P_ETH, P_IPV4, P_IPV6, P_TCP, P_UDP, P_ARP = 1, 2, 3, 4, 5, 8

def stats_settled(batch, summary, layers):
    """Per packet: (settled, L7 bits HTTP 1 / DNS 2 / SSL 4) for collectStats' counters (Common.h:83-104), from the
    parse flags: a packet is settled unless its chain stopped before an out-of-scope L2/L3 layer, its record is bad,
    or it has an L7 layer the parse did not classify (PCPPX_F_L7_KNOWN; restated in pcppx_oracle.c tcp_l7/udp_l7)."""
    fl = summary["flags"].astype(np.int64)
    settled = ((fl & (abi.F_NEEDS_HOST_PROTO | abi.F_OVERSIZE | abi.F_BAD_DESC)) == 0) & \
        (((fl & abi.F_NEEDS_HOST_L7) == 0) | ((fl & abi.F_L7_KNOWN) != 0))
    m = summary["proto_mask"].astype(np.uint64)
    bit = lambda p: ((m >> np.uint64(p)) & np.uint64(1)) != 0  # noqa: E731  (layers the parse built)
    l7 = ((((fl & abi.F_L7_HTTP) != 0) | bit(6) | bit(7)) * 1 | (((fl & abi.F_L7_DNS) != 0) | bit(13)) * 2 |
          (((fl & abi.F_L7_SSL) != 0) | bit(18)) * 4).astype(np.int32)
    return settled, l7


def oracle_filter(batch, summary, layers, spec: abi.MatchSpec, flow_table: dict | None = None):
    """Restatement of the FilterTraffic worker (AppWorkerThread.h:85-139; PacketMatchingEngine.h:43-107;
    Common.h:83-104) over parse records, in receive order. Pure Python: small batches only.
    Returns (matched u8[n], stats dict; the HTTP/DNS/SSL counters over the settled packets, see
    stats_settled). `flow_table` persists across calls."""
    ft = {} if flow_table is None else flow_table
    m_sip, m_dip = spec.src_ip != 0, spec.dst_ip != 0
    m_sp, m_dp = spec.src_port != 0, spec.dst_port != 0
    m_proto = spec.protocol in (P_TCP, P_UDP)
    st = {k: 0 for k in abi.STATS_FIELDS}
    matched = np.zeros(batch.n, dtype=np.uint8)
    data = batch.data
    settled, l7 = stats_settled(batch, summary, layers)
    for i in range(batch.n):
        mask = int(summary["proto_mask"][i])
        has = lambda p: (mask >> p) & 1  # noqa: E731
        st["packet_count"] += 1
        for key, p in (("eth_count", P_ETH), ("arp_count", P_ARP), ("ipv4_count", P_IPV4),
                       ("ipv6_count", P_IPV6), ("tcp_count", P_TCP), ("udp_count", P_UDP)):
            st[key] += has(p)
        if settled[i]:
            st["http_count"] += int(l7[i] & 1 != 0)
            st["dns_count"] += int(l7[i] & 2 != 0)
            st["tls_count"] += int(l7[i] & 4 != 0)
        else:
            st["needs_host_count"] += 1
        base = int(batch.offsets[i])
        nl = min(int(summary["n_layers"][i]), layers.shape[1])
        first = {}
        for k in range(nl):
            first.setdefault(int(layers[i, k]["proto"]), int(layers[i, k]["offset"]))

        def is_matched() -> bool:
            if m_sip or m_dip:
                if not has(P_IPV4):
                    return False
                o = base + first[P_IPV4]
                if m_sip and int.from_bytes(data[o + 12:o + 16].tobytes(), "little") != spec.src_ip:
                    return False
                if m_dip and int.from_bytes(data[o + 16:o + 20].tobytes(), "little") != spec.dst_ip:
                    return False
            if m_sp or m_dp:
                if has(P_TCP):
                    o = base + first[P_TCP]
                elif has(P_UDP):
                    o = base + first[P_UDP]
                else:
                    return False
                sp, dp = int(data[o]) << 8 | int(data[o + 1]), int(data[o + 2]) << 8 | int(data[o + 3])
                if m_sp and sp != spec.src_port:
                    return False
                if m_dp and dp != spec.dst_port:
                    return False
            if m_proto and not has(spec.protocol):
                return False
            return True

        h = int(summary["hash5"][i])
        if ft.get(h, False):
            ok = True
        else:
            ok = is_matched()
            if ok:
                ft[h] = True
                if has(P_TCP):
                    st["matched_tcp_flows"] += 1
                elif has(P_UDP):
                    st["matched_udp_flows"] += 1
        st["matched_packets"] += int(ok)
        matched[i] = ok
    return matched, st


def oracle_reasm(batch, summary, layers):
    """Restatement of the reassembly front ends (pcppx_reasm_device) from engine-format records
    (summary[n], layers[n, max_layers]) of the same batch: pcppx_reasm_info[n]."""
    n, ml = batch.n, layers.shape[1]
    info = np.zeros(max(n, 1), dtype=abi.REASM_DTYPE)
    s = np.ascontiguousarray(summary)
    lay = np.ascontiguousarray(layers)
    rec = abi.Records(s.ctypes.data, lay.ctypes.data)
    b = batch.c_batch()
    rc = oracle_lib().pcppx_oracle_reasm_batch(C.byref(b), C.byref(rec), ml, info.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"oracle reasm failed {rc}")
    return info[:n]


def ref_reasm(batch):
    """The real reference's IPReassembly / TcpReassembly first-sighting statuses and fragment fields per
    packet (oracle/ref_harness.cpp: pcppx_ref_reasm): pcppx_reasm_info[n]."""
    info = np.zeros(max(batch.n, 1), dtype=abi.REASM_DTYPE)
    b = batch.c_batch()
    rc = ref_lib().pcppx_ref_reasm(C.byref(b), info.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"reference reasm failed {rc}")
    return info[: batch.n]


def checksum(bufs: list[bytes]) -> int:
    arrs = [np.frombuffer(b + b"\0", np.uint8) for b in bufs]
    ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    lens = (C.c_uint32 * len(arrs))(*[len(b) for b in bufs])
    return oracle_lib().pcppx_oracle_checksum(ptrs, lens, len(arrs))


def fnv1(buf: bytes) -> int:
    a = np.frombuffer(buf + b"\0", np.uint8)
    return oracle_lib().pcppx_oracle_fnv1(a.ctypes.data, len(buf))


# ----- record comparison (engine contract, see pcppx_oracle.c header) -----
def compare_engine_to_reference(eng_sum, eng_lay, ref_sum, ref_lay) -> dict:
    """Check an engine-format record set (oracle or GPU) against reference records.

    Unflagged packets: every field equal. Flagged (NEEDS_HOST_*) packets: the emitted layers are an
    exact prefix of the reference chain. Returns counters; raises AssertionError on a violation.
    """
    n = len(eng_sum)
    flagged = (eng_sum["flags"] & abi.F_NEEDS_HOST) != 0
    ok = ~flagged
    stats = {"n": n, "flagged": int(flagged.sum()), "exact": int(ok.sum())}
    for f in ("hash5", "hash5_dir", "hash2", "flags", "n_layers", "l4_layer", "proto_mask",
              "ip_csum_calc", "ip_csum_stored", "l4_csum_calc", "l4_csum_stored"):
        bad = np.nonzero(ok & (eng_sum[f] != ref_sum[f]))[0]
        if len(bad):
            i = int(bad[0])
            raise AssertionError(f"field {f} differs on {len(bad)} unflagged packets; first #{i}: "
                                 f"engine={eng_sum[i]} ref={ref_sum[i]} layers engine={eng_lay[i]} ref={ref_lay[i]}")
    ml = eng_lay.shape[1]
    idx = np.arange(ml)[None, :]
    valid = idx < eng_sum["n_layers"][:, None]
    diff = np.zeros(eng_lay.shape, dtype=bool)
    for f in ("proto", "osi", "offset", "hdr_len", "data_len"):
        diff |= eng_lay[f] != ref_lay[f]
    bad = np.nonzero((diff & valid).any(axis=1))[0]
    if len(bad):
        i = int(bad[0])
        raise AssertionError(f"layer prefix differs on {len(bad)} packets; first #{i}: engine={eng_lay[i]} "
                             f"ref={ref_lay[i]} sum engine={eng_sum[i]} ref={ref_sum[i]}")
    shorter = flagged & (eng_sum["n_layers"] > ref_sum["n_layers"])
    if shorter.any():
        i = int(np.nonzero(shorter)[0][0])
        raise AssertionError(f"flagged packet #{i} has more layers than the reference")
    # NEEDS_HOST_L7 packets whose whole reference chain is visible and holds no IPv4 / IPv6 / TCP / UDP layer past the
    # engine's prefix: hash5Tuple / hash2Tuple (first IP, last TCP else UDP: PacketUtils.cpp:139-245), the port layer
    # and both checksums come from layers the engine built, so they are exact as well
    l7only = flagged & ((eng_sum["flags"] & (abi.F_NEEDS_HOST & ~abi.F_NEEDS_HOST_L7)) == 0)
    past = (idx >= eng_sum["n_layers"][:, None]) & (idx < ref_sum["n_layers"][:, None]) & \
        np.isin(ref_lay["proto"], (2, 3, 4, 5))
    l7exact = l7only & (ref_sum["n_layers"] < ml) & ~past.any(axis=1)
    for f in ("hash5", "hash5_dir", "hash2", "l4_layer", "ip_csum_calc", "ip_csum_stored", "l4_csum_calc",
              "l4_csum_stored"):
        bad = np.nonzero(l7exact & (eng_sum[f] != ref_sum[f]))[0]
        if len(bad):
            i = int(bad[0])
            raise AssertionError(f"field {f} differs on {len(bad)} NEEDS_HOST_L7 packets; first #{i}: "
                                 f"engine={eng_sum[i]} ref={ref_sum[i]} layers engine={eng_lay[i]} ref={ref_lay[i]}")
    stats["l7_flagged_exact_5tuple"] = int(l7exact.sum())
    return stats


# protocols the engine builds itself (include/pcppx.h: everything else is a host layer); HTTPRequest /
# HTTPResponse (6/7), DNS (13), SSL (18), SSH (35) and MySQL (63) as a classified first L7 layer and the layers behind it
ENGINE_PROTOS = (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 13, 14, 15, 16, 17, 18, 19, 21, 25, 26, 30, 32, 33, 35, 44, 47, 52, 58,
                 63)  # 47 NFLOG, 58 Cisco HDLC: first layers built since round 6


# TcpLayer::parseNextLayer's trigger ports (TcpLayer.cpp:372-491; pcppx_oracle.c tcp_l7_port), HTTP's (HttpLayer.h:74-77)
# and SSL's (SSLLayer.h:488-510)
TCP_L7_PORTS = frozenset((80, 8080, 5060, 5061, 179, 22, 53, 5353, 5355, 23, 21, 20, 13400, 3496, 30490, 102, 25, 587,
                          389, 5432, 3306, 2123, 502, 443, 261, 448, 465, 563, 614, 636, 989, 990, 992, 993, 994, 995))
HTTP_PORTS = frozenset((80, 8080))
SSL_PORTS = frozenset((443, 261, 448, 465, 563, 614, 636, 989, 990, 992, 993, 994, 995))


def _mysql_behind_earlier_dissector(batch, i: int, lay) -> bool:
    """Packet i's last TCP layer (reference records `lay`, one packet) has port 3306 on one side and on the other a
    trigger port whose dissector comes ahead of MySQL's in TcpLayer::parseNextLayer and has a validity rule of its own
    (not 3306, GTPv2 2123, Modbus 502, HTTP or SSL): the only case where the reference may fall through to MySQL after
    the engine left the payload to the host (pcppx_oracle.c tcp_l7, the MySQL rule)."""
    tcp = [k for k in range(len(lay)) if lay["proto"][k] == 4]
    if not tcp:
        return False
    off = int(lay["offset"][tcp[-1]])
    pkt = batch.packet(i)
    if off + 4 > len(pkt):
        return False
    sp, dp = int.from_bytes(pkt[off:off + 2], "big"), int.from_bytes(pkt[off + 2:off + 4], "big")
    if 3306 not in (sp, dp):
        return False
    o = dp if sp == 3306 else sp
    return o not in (3306, 2123, 502) and o in TCP_L7_PORTS and o not in HTTP_PORTS and o not in SSL_PORTS


def check_flag_contract(eng_sum, ref_sum, ref_lay, batch=None) -> dict:
    """The NEEDS_HOST flags against the reference chain (records with max_layers >= 1):
      - every packet whose reference chain holds a layer the engine does not build is flagged
        (NEEDS_HOST_L7 / NEEDS_HOST_PROTO, or not parsed at all: OVERSIZE / BAD_DESC);
      - a flagged packet whose reference chain holds no such layer is one where the host's dissector, at the
        point the engine stopped, built nothing or fell back to a Payload layer, or (port 3306 beside another trigger
        port) the earlier dissector declined and the chain fell through to MySQL -- the engine cannot tell without
        that dissector's own validity rules: the reference layer at index n_layers is GenericPayload or absent, or
        MySQL exactly where the packet's ports are 3306 beside such a trigger port (checked from the bytes: `batch`
        is required whenever a reference chain continues with MySQL).
    Returns counters {flagged, foreign, payload_fallback}."""
    host = (eng_sum["flags"] & (abi.F_NEEDS_HOST_L7 | abi.F_NEEDS_HOST_PROTO)) != 0
    unparsed = (eng_sum["flags"] & (abi.F_OVERSIZE | abi.F_BAD_DESC)) != 0
    ml = ref_lay.shape[1]
    rn = np.minimum(ref_sum["n_layers"].astype(np.int64), ml)
    valid = np.arange(ml)[None, :] < rn[:, None]
    foreign = (valid & ~np.isin(ref_lay["proto"], ENGINE_PROTOS)).any(axis=1)
    miss = np.nonzero(foreign & ~host & ~unparsed)[0]
    if len(miss):
        i = int(miss[0])
        raise AssertionError(f"{len(miss)} packets hold a host layer but are not flagged; first #{i}: "
                             f"engine={eng_sum[i]} ref={ref_lay[i][: rn[i]]}")
    over = np.nonzero(host & ~foreign)[0]
    en = eng_sum["n_layers"][over].astype(np.int64)
    nxt = np.where(en < rn[over], ref_lay["proto"][over, np.minimum(en, ml - 1)], 25)
    mysql = over[nxt == 63]
    ok_mysql = np.array([batch is not None and _mysql_behind_earlier_dissector(batch, int(i), ref_lay[i][: rn[i]])
                         for i in mysql], dtype=bool)
    bad = np.concatenate([over[(nxt != 25) & (nxt != 63)], mysql[~ok_mysql]]) if len(mysql) else \
        over[(nxt != 25) & (nxt != 63)]
    if len(bad):
        i = int(bad[0])
        raise AssertionError(f"{len(bad)} flagged packets whose reference chain continues with an engine layer; "
                             f"first #{i}: engine={eng_sum[i]} ref={ref_lay[i][: rn[i]]}")
    # the first L7 layer's class (PCPPX_F_L7_*) against the reference chain's HTTPRequest/HTTPResponse (6/7),
    # SSL (18) and DNS (13) layers
    fl = eng_sum["flags"]
    known = ((fl & abi.F_NEEDS_HOST_L7) != 0) & ((fl & abi.F_L7_KNOWN) != 0)
    m = ref_sum["proto_mask"].astype(np.uint64)
    bit = lambda p: ((m >> np.uint64(p)) & np.uint64(1)).astype(bool)  # noqa: E731
    for name, f, has in (("HTTP", abi.F_L7_HTTP, bit(6) | bit(7)), ("SSL", abi.F_L7_SSL, bit(18)),
                         ("DNS", abi.F_L7_DNS, bit(13))):
        bad = np.nonzero(known & (((fl & f) != 0) != has))[0]
        if len(bad):
            i = int(bad[0])
            raise AssertionError(f"L7 class {name} differs on {len(bad)} packets; first #{i}: engine={eng_sum[i]} "
                                 f"ref={ref_lay[i][: rn[i]]}")
    return {"flagged": int(host.sum()), "foreign": int(foreign.sum()), "payload_fallback": int(len(over)),
            "l7_known": int(known.sum())}


def compare_exact(a_sum, a_lay, b_sum, b_lay) -> None:
    """Bit-exact equality of two engine-format record sets (GPU vs oracle), all packets."""
    for f in a_sum.dtype.names:
        bad = np.nonzero(a_sum[f] != b_sum[f])[0]
        if len(bad):
            i = int(bad[0])
            raise AssertionError(f"summary.{f} differs on {len(bad)} packets; first #{i}: {a_sum[i]} vs {b_sum[i]}")
    ml = a_lay.shape[1]
    valid = np.arange(ml)[None, :] < a_sum["n_layers"][:, None]
    for f in a_lay.dtype.names:
        bad = np.nonzero(((a_lay[f] != b_lay[f]) & valid).any(axis=1))[0]
        if len(bad):
            i = int(bad[0])
            raise AssertionError(f"layers.{f} differs on {len(bad)} packets; first #{i}: {a_lay[i]} vs {b_lay[i]}")
