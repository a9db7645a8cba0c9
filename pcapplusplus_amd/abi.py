"""ctypes/numpy mirror of include/pcppx.h (the engine's C ABI) and the loader of libpcppx.so.

The loader fails loudly when the HIP engine library is missing: there is no CPU fallback in the
product path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
ENGINE_SO = PKG_DIR / "libpcppx.so"

ABI_VERSION = 7
MAX_LAYERS = 16
MAX_CAPLEN = 65535
WINDOW_DEFAULT, WINDOW_DEEP, WINDOW_SHORT = 0, 1, 2  # pcppx_opts.window (PCPPX_WINDOW_*)
LAYOUT_FIXED, LAYOUT_PACKED, LAYOUT_DENSE = 0, 1, 2  # pcppx_opts.layout (PCPPX_LAYOUT_*); DENSE: host path
PACKED_MAX_LAYERS = 12
TILE = 64  # packets per tile of the PACKED layout

# error codes
OK, E_INVAL, E_NODEV, E_HIP, E_NOMEM, E_LINKTYPE = 0, -1, -2, -3, -4, -5

# summary flags
F_NEEDS_HOST_L7 = 0x0001
F_NEEDS_HOST_PROTO = 0x0002
F_DEPTH_OVERFLOW = 0x0004
F_OVERSIZE = 0x0008
F_IP_CSUM = 0x0010
F_IP_CSUM_OK = 0x0020
F_L4_CSUM = 0x0040
F_L4_CSUM_OK = 0x0080
F_TRAILER = 0x0100
F_BAD_DESC = 0x0200
F_L7_KNOWN = 0x0400
F_L7_HTTP = 0x0800
F_L7_SSL = 0x1000
F_L7_DNS = 0x2000
F_NEEDS_HOST = F_NEEDS_HOST_L7 | F_NEEDS_HOST_PROTO | F_OVERSIZE | F_BAD_DESC

# pcpp::LinkLayerType values used here (Packet++/header/RawPacket.h:24-178)
LINKTYPE_NULL = 0
LINKTYPE_ETHERNET = 1
LINKTYPE_DLT_RAW1 = 12
LINKTYPE_DLT_RAW2 = 14
LINKTYPE_RAW = 101
LINKTYPE_LINUX_SLL = 113
LINKTYPE_IPV4 = 228
LINKTYPE_IPV6 = 229

SUMMARY_DTYPE = np.dtype(
    [
        ("hash5", "<u4"),
        ("hash5_dir", "<u4"),
        ("hash2", "<u4"),
        ("flags", "<u2"),
        ("n_layers", "u1"),
        ("l4_layer", "u1"),
        ("proto_mask", "<u8"),
        ("ip_csum_calc", "<u2"),
        ("ip_csum_stored", "<u2"),
        ("l4_csum_calc", "<u2"),
        ("l4_csum_stored", "<u2"),
    ]
)
BRIEF_DTYPE = np.dtype(SUMMARY_DTYPE.descr[:6])  # pcppx_brief (ABI 7): the summary's first 16 bytes
LAYER_DTYPE = np.dtype(
    [("proto", "u1"), ("osi", "u1"), ("offset", "<u2"), ("hdr_len", "<u2"), ("data_len", "<u2")]
)
REASM_DTYPE = np.dtype(
    [("ip_key", "<u4"), ("frag_id", "<u4"), ("frag_offset", "<u2"), ("ip_status", "u1"), ("tcp_status", "u1"),
     ("tcp_payload", "<u4")]
)
TUPLE_DTYPE = np.dtype(
    [("src_ip", "u1", (16,)), ("dst_ip", "u1", (16,)), ("src_port", "<u2"), ("dst_port", "<u2"), ("ip_version", "u1"),
     ("ip_proto", "u1"), ("l4_proto", "u1"), ("has_5tuple", "u1"), ("hash5", "<u4"), ("flags", "<u2"),
     ("n_layers", "u1"), ("reserved", "u1")]
)
assert SUMMARY_DTYPE.itemsize == 32 and LAYER_DTYPE.itemsize == 8 and REASM_DTYPE.itemsize == 16
assert BRIEF_DTYPE.itemsize == 16
assert TUPLE_DTYPE.itemsize == 48

# pcppx_records.proto_stats words (PCPPX_PS_*): PacketStats::collectStats, Common.h:83-104
PROTO_STATS = 16
PROTO_STATS_FIELDS = ("packet_count", "eth_count", "arp_count", "ipv4_count", "ipv6_count", "tcp_count", "udp_count",
                      "http_count", "dns_count", "tls_count", "needs_host_count")

# pcppx_reasm_info status codes (low nibble) and flags
IPR_NON_IP, IPR_NON_FRAGMENT, IPR_MALFORMED, IPR_FRAGMENT, IPR_HOST = 0, 1, 2, 3, 15
IPR_F_FIRST, IPR_F_LAST, IPR_F_IPV6 = 0x10, 0x20, 0x40
TCPR_NON_IP, TCPR_NON_TCP, TCPR_NO_DATA, TCPR_DATA, TCPR_HOST = 0, 1, 2, 3, 15
TCPR_F_FIN, TCPR_F_SYN, TCPR_F_RST = 0x10, 0x20, 0x40


class Batch(C.Structure):
    _fields_ = [
        ("data", C.c_void_p),
        ("offsets", C.c_void_p),
        ("caplens", C.c_void_p),
        ("data_len", C.c_uint64),
        ("n", C.c_uint32),
        ("linktype", C.c_uint16),
        ("reserved", C.c_uint16),
    ]


class Opts(C.Structure):
    _fields_ = [
        ("parse_until_family", C.c_uint32),
        ("parse_until_osi", C.c_uint8),
        ("want_checksums", C.c_uint8),
        ("max_layers", C.c_uint8),
        ("window", C.c_uint8),
        ("layout", C.c_uint8),
        ("reserved", C.c_uint8 * 3),
    ]


class Records(C.Structure):
    _fields_ = [("summary", C.c_void_p), ("layers", C.c_void_p), ("flow_keys", C.c_void_p), ("tuples", C.c_void_p),
                ("proto_stats", C.c_void_p), ("layout", C.c_uint8), ("reserved", C.c_uint8 * 7),
                ("brief", C.c_void_p), ("layers_written", C.c_uint64)]


class MatchSpec(C.Structure):
    """pcppx_match_spec: PacketMatchingEngine's criteria (PacketMatchingEngine.h:28-41)."""
    _fields_ = [("src_ip", C.c_uint32), ("dst_ip", C.c_uint32), ("src_port", C.c_uint16), ("dst_port", C.c_uint16),
                ("protocol", C.c_uint8), ("reserved", C.c_uint8 * 3)]


STATS_FIELDS = ("packet_count", "eth_count", "arp_count", "ipv4_count", "ipv6_count", "tcp_count", "udp_count",
                "http_count", "dns_count", "tls_count", "matched_tcp_flows", "matched_udp_flows", "matched_packets",
                "needs_host_count", "flow_table_full")


class PacketStats(C.Structure):
    """pcppx_packet_stats: PacketStats (Examples/DpdkExample-FilterTraffic/Common.h:57-142)."""
    _fields_ = [(f, C.c_uint64) for f in STATS_FIELDS]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f in STATS_FIELDS}


def ipv4_to_int(dotted: str) -> int:
    """IPv4Address::toInt(): the address bytes in memory order read as a little-endian u32."""
    b = bytes(int(x) for x in dotted.split("."))
    return int.from_bytes(b, "little")


def make_opts(parse_until_family: int = 0, parse_until_osi: int = 8, want_checksums: bool = True,
              max_layers: int = MAX_LAYERS, window: int = 0, layout: int = LAYOUT_FIXED) -> Opts:
    """pcpp::PacketParseOptions defaults (Packet++/header/Packet.h:17-37) + output selection; window:
    WINDOW_DEFAULT / WINDOW_DEEP / WINDOW_SHORT (the header window the parse gathers: a speed choice, records
    identical; DEEP: two rounds for checksum launches, SHORT: one 96-B round for parse-only launches); layout: LAYOUT_FIXED /
    LAYOUT_PACKED (the layer entries, bit for bit the same; unpack_layers)."""
    if not 0 <= max_layers <= MAX_LAYERS:
        raise ValueError(f"max_layers must be in [0, {MAX_LAYERS}]")
    if window not in (WINDOW_DEFAULT, WINDOW_DEEP, WINDOW_SHORT):
        raise ValueError("window must be WINDOW_DEFAULT, WINDOW_DEEP or WINDOW_SHORT")
    if layout not in (LAYOUT_FIXED, LAYOUT_PACKED, LAYOUT_DENSE) or \
            (layout == LAYOUT_PACKED and max_layers > PACKED_MAX_LAYERS):
        raise ValueError(f"layout must be LAYOUT_FIXED, LAYOUT_DENSE (host path), or LAYOUT_PACKED with max_layers <= "
                         f"{PACKED_MAX_LAYERS}")
    o = Opts(parse_until_family, parse_until_osi, 1 if want_checksums else 0, max_layers, window)
    o.layout = layout
    return o


def packed_positions(n_layers: np.ndarray, max_layers: int) -> np.ndarray:
    """Start entry of every packet's chain in a PACKED layer array (include/pcppx.h PCPPX_LAYOUT_PACKED): the tile's
    base 64 * t * max_layers plus the chains of the packets before it in its 64-packet tile."""
    cnt = np.minimum(n_layers.astype(np.int64), max_layers)
    n = len(cnt)
    tile = np.arange(n) // TILE
    csum = np.cumsum(cnt) - cnt  # exclusive prefix over the whole batch
    first = tile * TILE
    return tile * TILE * max_layers + csum - csum[first] if n else csum


def unpack_layers(summary: np.ndarray, packed: np.ndarray, max_layers: int) -> np.ndarray:
    """PACKED layer entries -> the FIXED [n, max_layers] array (entries past a chain zero)."""
    n = len(summary)
    out = np.zeros((n, max_layers), dtype=LAYER_DTYPE)
    if n == 0 or max_layers == 0:
        return out
    cnt = np.minimum(summary["n_layers"].astype(np.int64), max_layers)
    start = packed_positions(summary["n_layers"], max_layers)
    flat = packed.reshape(-1)
    for k in range(max_layers):
        m = cnt > k
        out[m, k] = flat[start[m] + k]
    return out


def dense_positions(n_layers: np.ndarray, max_layers: int) -> np.ndarray:
    """Start entry of every packet's chain in a DENSE layer array (PCPPX_LAYOUT_DENSE): the chains of the packets
    before it, whole batch."""
    cnt = np.minimum(n_layers.astype(np.int64), max_layers)
    return np.cumsum(cnt) - cnt


def unpack_dense(n_layers: np.ndarray, dense: np.ndarray, max_layers: int) -> np.ndarray:
    """DENSE layer entries -> the FIXED [n, max_layers] array (entries past a chain zero)."""
    n = len(n_layers)
    out = np.zeros((n, max_layers), dtype=LAYER_DTYPE)
    if n == 0 or max_layers == 0:
        return out
    cnt = np.minimum(n_layers.astype(np.int64), max_layers)
    start = dense_positions(n_layers, max_layers)
    flat = dense.reshape(-1)
    for k in range(max_layers):
        m = cnt > k
        out[m, k] = flat[start[m] + k]
    return out


def chain_proto_mask(fixed: np.ndarray, n_layers: np.ndarray) -> np.ndarray:
    """pcppx_chain_proto_mask over FIXED rows: Packet::isPacketOfType's mask from the recorded chain."""
    n, ml = fixed.shape
    k = np.arange(ml)[None, :] < np.minimum(n_layers.astype(np.int64), ml)[:, None]
    bits = np.where(k & (fixed["proto"] < 64), np.left_shift(np.uint64(1), fixed["proto"].astype(np.uint64)),
                    np.uint64(0))
    return np.bitwise_or.reduce(bits, axis=1) if ml else np.zeros(n, np.uint64)


def _declare(lib: C.CDLL) -> C.CDLL:
    P = C.c_void_p
    lib.pcppx_abi_version.restype = C.c_int
    lib.pcppx_strerror.restype = C.c_char_p
    lib.pcppx_strerror.argtypes = [C.c_int]
    lib.pcppx_device_count.argtypes = [C.POINTER(C.c_int)]
    lib.pcppx_runtime_info.argtypes = [C.c_int, C.c_char_p, C.c_size_t]
    lib.pcppx_runtime_info.restype = C.c_int
    lib.pcppx_open.argtypes = [C.c_int, C.POINTER(P)]
    lib.pcppx_close.argtypes = [P]
    lib.pcppx_close.restype = None
    lib.pcppx_sync.argtypes = [P]
    lib.pcppx_ctx_stream.argtypes = [P]
    lib.pcppx_ctx_stream.restype = P
    lib.pcppx_default_opts.argtypes = [C.POINTER(Opts)]
    lib.pcppx_default_opts.restype = None
    lib.pcppx_parse_batch_device.argtypes = [P, C.POINTER(Batch), C.POINTER(Opts), C.POINTER(Records), P]
    lib.pcppx_parse_batch_host.argtypes = [P, C.POINTER(Batch), C.POINTER(Opts), C.POINTER(Records)]
    lib.pcppx_flow_count_device.argtypes = [P, P, P, C.c_uint32, P, P, P, C.c_uint32, P, P]
    lib.pcppx_flow_count_keys_device.argtypes = [P, P, P, C.c_uint32, P, P, P, C.c_uint32, P, P]
    lib.pcppx_flow_count_keys_device.restype = C.c_int
    lib.pcppx_filter_device.argtypes = [P, C.POINTER(Batch), C.POINTER(Records), C.c_uint8, C.POINTER(MatchSpec),
                                        C.c_uint64, P, P, C.c_uint32, P, P, P]
    lib.pcppx_filter_device.restype = C.c_int
    lib.pcppx_reasm_device.argtypes = [P, C.POINTER(Batch), C.POINTER(Records), C.c_uint8, P, P]
    lib.pcppx_reasm_device.restype = C.c_int
    lib.pcppx_parse_batch_device_reasm.argtypes = [P, C.POINTER(Batch), C.POINTER(Opts), C.POINTER(Records), P, P]
    lib.pcppx_parse_batch_device_reasm.restype = C.c_int
    lib.pcppx_filter_reset.argtypes = [P, C.c_uint32]
    lib.pcppx_filter_reset.restype = C.c_int
    lib.pcppx_filter_batch_host.argtypes = [P, C.POINTER(Batch), C.POINTER(MatchSpec), P, C.POINTER(PacketStats)]
    lib.pcppx_filter_batch_host.restype = C.c_int
    lib.pcppx_pcap_open.argtypes = [C.c_char_p, C.POINTER(P)]
    lib.pcppx_pcap_open.restype = C.c_int
    lib.pcppx_pcap_linktype.argtypes = [P]
    lib.pcppx_pcap_linktype.restype = C.c_uint32
    lib.pcppx_pcap_read_batch.argtypes = [P, P, C.c_uint64, P, P, P, C.c_uint32, C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_uint64)]
    lib.pcppx_pcap_read_batch.restype = C.c_int
    lib.pcppx_pcap_read_batch_ex.argtypes = [P, P, C.c_uint64, P, P, P, P, C.c_uint32, C.POINTER(C.c_uint32),
                                             C.POINTER(C.c_uint64)]
    lib.pcppx_pcap_read_batch_ex.restype = C.c_int
    lib.pcppx_pcap_map_batch.argtypes = [P, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), P, P, P, P, C.c_uint32,
                                         C.POINTER(C.c_uint32)]
    lib.pcppx_pcap_map_batch.restype = C.c_int
    lib.pcppx_pcap_close.argtypes = [P]
    lib.pcppx_pcap_close.restype = None
    lib.pcppx_host_alloc.argtypes = [C.c_size_t]
    lib.pcppx_host_alloc.restype = P
    lib.pcppx_host_free.argtypes = [P]
    lib.pcppx_host_free.restype = None
    lib.pcppx_unpack_layers.argtypes = [P, P, C.c_uint64, C.c_uint32, P]
    lib.pcppx_unpack_layers.restype = C.c_int
    lib.pcppx_window_choice.argtypes = [P, C.c_int, C.POINTER(C.c_int)]
    lib.pcppx_window_choice.restype = C.c_int
    lib.pcppx_unpack_layers_brief.argtypes = [P, P, C.c_uint64, C.c_uint32, P]
    lib.pcppx_unpack_layers_brief.restype = C.c_int
    for name in ("pcppx_device_count", "pcppx_open", "pcppx_sync", "pcppx_parse_batch_device",
                 "pcppx_parse_batch_host", "pcppx_flow_count_device"):
        getattr(lib, name).restype = C.c_int
    return lib


_ENGINE: C.CDLL | None = None

# every symbol include/pcppx.h declares
EXPORTED_SYMBOLS = (
    "pcppx_abi_version", "pcppx_strerror", "pcppx_device_count", "pcppx_runtime_info", "pcppx_open", "pcppx_close",
    "pcppx_sync", "pcppx_ctx_stream", "pcppx_default_opts", "pcppx_parse_batch_device", "pcppx_parse_batch_host",
    "pcppx_flow_count_device", "pcppx_flow_count_keys_device", "pcppx_filter_device", "pcppx_filter_reset", "pcppx_filter_batch_host", "pcppx_reasm_device", "pcppx_parse_batch_device_reasm", "pcppx_pcap_open", "pcppx_pcap_linktype",
    "pcppx_pcap_read_batch", "pcppx_pcap_read_batch_ex", "pcppx_pcap_map_batch", "pcppx_pcap_close", "pcppx_host_alloc", "pcppx_host_free",
    "pcppx_unpack_layers", "pcppx_unpack_layers_brief", "pcppx_window_choice",
)


def load_engine() -> C.CDLL:
    """Load the HIP engine (pcapplusplus_amd/libpcppx.so). Raises if it has not been built."""
    global _ENGINE
    if _ENGINE is None:
        if not ENGINE_SO.exists():
            raise RuntimeError(
                f"HIP engine library {ENGINE_SO} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`"
                " (or `make -C pcapplusplus_amd/csrc`). There is no CPU fallback.")
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7. Importing torch first makes
        # the engine bind to that same runtime (matched by SONAME), so torch tensors/streams and the
        # engine's kernels share one device context.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = _declare(C.CDLL(str(ENGINE_SO)))
        if lib.pcppx_abi_version() != ABI_VERSION:
            raise RuntimeError("libpcppx.so ABI version mismatch")
        _ENGINE = lib
    return _ENGINE


def runtime_info(device: int = 0) -> str:
    buf = C.create_string_buffer(256)
    load_engine().pcppx_runtime_info(device, buf, 256)
    return buf.value.decode()


def check(rc: int, what: str = "pcppx") -> None:
    if rc != OK:
        msg = load_engine().pcppx_strerror(rc).decode() if _ENGINE is not None else str(rc)
        raise RuntimeError(f"{what} failed: {msg} ({rc})")


def ptr(a) -> int:
    """Data pointer of a numpy array or torch tensor."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


__all__ = [n for n in dir() if not n.startswith("_")]
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
