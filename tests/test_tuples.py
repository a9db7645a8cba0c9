"""The 5-tuple extract (pcppx_records.tuples, include/pcppx.h pcppx_tuple) and the collectStats counters
(pcppx_records.proto_stats).

CPU: the restatement's extract (oracle_parse_tuples) equals the reference's own accessors -- frozen from the real
Packet++ in tests/golden/tuples/ref_tuples.npz (tools/make_golden_tuples.py), and live where oracle/_ref is built --
on every golden set; hash5Tuple recomputed from the extracted fields equals the summary's hash5 (the tuple holds exactly
the bytes hashed, PacketUtils.cpp:139-210).
GPU: the device extract equals the restatement bit for bit (every field, flags and n_layers included) on every golden
set, crafted deep / L7 stacks and BASELINE config 2 at its full 1M packets; the device's collectStats counters equal
the restatement's and, on the reference's example.pcap / example2.pcap, the reference FilterTraffic worker's own.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, golden_files, load_golden
from pcapplusplus_amd import abi, synth

REF_TUPLES = GOLDEN / "tuples" / "ref_tuples.npz"


def fnv1(data: bytes) -> int:
    h = 2166136261
    for b in data:
        h = (h * 16777619) & 0xFFFFFFFF
        h ^= b
    return h


def hash5_from_tuple(t, direction_unique: bool = False) -> int:
    """hash5Tuple (PacketUtils.cpp:139-210) recomputed from one extracted tuple alone: the ports as they sit in the
    header compared as in-memory u16 (:169-173), then -- equal ports only -- the addresses (:183-185, :197-199); one
    srcPosition orders both pairs; the IP layer's protocol byte last."""
    if not t["has_5tuple"]:
        return 0
    sp = int(t["src_port"]).to_bytes(2, "big")
    dp = int(t["dst_port"]).to_bytes(2, "big")
    na = 4 if t["ip_version"] == 4 else 16
    si, di = bytes(t["src_ip"][:na]), bytes(t["dst_ip"][:na])
    raw_sp, raw_dp = int.from_bytes(sp, "little"), int.from_bytes(dp, "little")
    swap = not direction_unique and raw_dp < raw_sp
    if not direction_unique and raw_sp == raw_dp:
        swap = int.from_bytes(di, "little") < int.from_bytes(si, "little") if na == 4 else di < si
    ports = dp + sp if swap else sp + dp
    ips = di + si if swap else si + di
    return fnv1(ports + ips + bytes([int(t["ip_proto"])]))


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.stem)
def test_oracle_tuples_match_reference(path):
    batch, _ = load_golden(path)
    s, _, t = oracle.oracle_parse_tuples(batch, abi.make_opts(0, 8, False, 16))
    frozen = np.load(REF_TUPLES, allow_pickle=False)[path.stem]
    st = oracle.compare_tuples(t, frozen, s)
    assert st["n"] == batch.n
    if oracle.ref_available():
        oracle.compare_tuples(t, oracle.ref_tuples(batch), s)
    # the summary fields the tuple repeats
    assert np.array_equal(t["hash5"], s["hash5"]) and np.array_equal(t["flags"], s["flags"])
    assert np.array_equal(t["n_layers"], s["n_layers"])


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.stem)
def test_tuple_fields_are_the_hashed_bytes(path):
    batch, _ = load_golden(path)
    s, _, t = oracle.oracle_parse_tuples(batch, abi.make_opts(0, 8, False, 16))
    ok = (s["flags"] & abi.F_NEEDS_HOST) == 0
    for i in np.nonzero(ok)[0][:3000]:
        assert hash5_from_tuple(t[i]) == int(s["hash5"][i]), i
        assert hash5_from_tuple(t[i], True) == int(s["hash5_dir"][i]), i


def test_oracle_proto_stats_match_reference_worker():
    """collectStats totals of the restatement's summaries == the reference FilterTraffic worker's PacketStats
    (ref_filter, an empty PacketMatchingEngine) on example.pcap."""
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built")
    batch, _ = load_golden(GOLDEN / "capture_example.npz")
    s, _ = oracle.oracle_parse(batch, abi.make_opts(0, 8, False, 16))
    _, ref = oracle.ref_filter(batch, oracle.make_spec())
    mine = oracle.proto_stats(s)
    assert mine["needs_host_count"] == 0
    for k in abi.PROTO_STATS_FIELDS[:-1]:
        assert mine[k] == ref[k], k


def test_packed_layout_decode_roundtrip():
    """abi.unpack_layers(packed_positions) inverts the PACKED layout (include/pcppx.h) built in numpy from FIXED rows."""
    batch = synth.config(5, 1000)
    ml = 12
    s, lay = oracle.oracle_parse(batch, abi.make_opts(0, 8, False, ml))
    cnt = np.minimum(s["n_layers"].astype(np.int64), ml)
    packed = np.zeros(batch.n * ml, dtype=abi.LAYER_DTYPE)
    pos = abi.packed_positions(s["n_layers"], ml)
    for i in range(batch.n):
        packed[pos[i]:pos[i] + cnt[i]] = lay[i, :cnt[i]]
        t = i // abi.TILE
        assert pos[i] >= t * abi.TILE * ml and pos[i] + cnt[i] <= (t + 1) * abi.TILE * ml
    back = abi.unpack_layers(s, packed, ml)
    valid = np.arange(ml)[None, :] < cnt[:, None]
    assert (back[valid] == lay[valid]).all()


# ---------------------------------------------------------------- GPU ----------------------------------------------
def _device(engine, batch, opts, summary=True, tuples=True, stats=True):
    from pcapplusplus_amd.engine import parse_on_device_ex

    return parse_on_device_ex(engine, batch, opts, summary=summary, tuples=tuples, proto_stats=stats)


@pytest.mark.gpu
@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.stem)
def test_gpu_tuples_and_stats_golden(engine, path):
    batch, variants = load_golden(path)
    frozen = np.load(REF_TUPLES, allow_pickle=False)[path.stem]
    for v, (opts, rsum, rlay) in variants.items():
        g = _device(engine, batch, opts)
        os_, _, ot = oracle.oracle_parse_tuples(batch, opts)
        assert g["tuples"].tobytes() == ot.tobytes(), v
        assert g["proto_stats"] == oracle.proto_stats(os_), v
        assert not g["proto_stats_raw"][len(abi.PROTO_STATS_FIELDS):].any()
        if v == "full":
            oracle.compare_tuples(g["tuples"], frozen, g["summary"])
    # tuples alone (no summary, no layers): the same extract
    g = _device(engine, batch, abi.make_opts(0, 8, False, 0), summary=False, stats=False)
    _, _, ot = oracle.oracle_parse_tuples(batch, abi.make_opts(0, 8, False, 0))
    assert g["tuples"].tobytes() == ot.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("gaps", [False, True])
def test_gpu_tuples_crafted(engine, gaps):
    from mutate import as_batch, crafted, crafted_l7

    b = as_batch(crafted() + crafted_l7(), gaps=gaps, seed=23)
    for opts in (abi.make_opts(), abi.make_opts(0, 8, False, 0), abi.make_opts(4, 8, True, 16),
                 abi.make_opts(0, 8, True, 12, abi.WINDOW_DEEP)):
        g = _device(engine, b, opts)
        os_, _, ot = oracle.oracle_parse_tuples(b, opts)
        assert g["tuples"].tobytes() == ot.tobytes()
        assert g["proto_stats"] == oracle.proto_stats(os_)


@pytest.mark.gpu
def test_gpu_config2_full_size_tuples(engine):
    """BASELINE config 2 at its full 1M 64-B packets: the bench's own output (tuples only, no summary) equals the
    restatement's extract on every packet, and every packet carries a 5-tuple."""
    b = synth.config(2, 1_000_000)
    opts = abi.make_opts(0, 8, False, 0)
    g = _device(engine, b, opts, summary=False, stats=False)
    _, _, ot = oracle.oracle_parse_tuples(b, opts, threads=8)
    assert g["tuples"].tobytes() == ot.tobytes()
    assert (g["tuples"]["has_5tuple"] == 1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["example.pcap", "example2.pcap"])
def test_gpu_proto_stats_equal_reference_worker(engine, name):
    """collectStats (Common.h:83-104) on the device, over the reference's own captures, equals the reference
    FilterTraffic worker's PacketStats."""
    from test_examples import capture

    batch, _ = capture(name)
    g = _device(engine, batch, abi.make_opts(0, 8, False, 0), tuples=False)
    st = g["proto_stats"]
    if oracle.ref_available():
        _, ref = oracle.ref_filter(batch, oracle.make_spec())
        for k in abi.PROTO_STATS_FIELDS[:-1]:
            assert st[k] == ref[k], (k, st[k], ref[k])
    s, _ = oracle.oracle_parse(batch, abi.make_opts(0, 8, False, 16))
    assert st == oracle.proto_stats(s)
    assert st["needs_host_count"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,ml,csum", [(3, 8, True), (5, 12, False), (5, 12, True), (4, 5, False), (3, 1, True)])
def test_gpu_packed_layout(engine, cfg, ml, csum):
    """PCPPX_LAYOUT_PACKED: the chains dense per 64-packet tile decode (abi.unpack_layers) to exactly the FIXED
    layout's entries; the summary, tuples and stats are unchanged; a gapped batch (generic-walk lanes write through
    their fixed slot and are moved into the run) and every golden set too."""
    from mutate import as_batch

    b = synth.config(cfg, 100_000)
    fixed = _device(engine, b, abi.make_opts(0, 8, csum, ml))
    packed = _device(engine, b, abi.make_opts(0, 8, csum, ml, layout=abi.LAYOUT_PACKED))
    oracle.compare_exact(packed["summary"], packed["layers"], fixed["summary"], fixed["layers"])
    assert packed["tuples"].tobytes() == fixed["tuples"].tobytes()
    assert packed["proto_stats"] == fixed["proto_stats"]
    g = as_batch([b.packet(i) for i in range(20_000)], gaps=True, seed=cfg)
    gp = _device(engine, g, abi.make_opts(0, 8, csum, ml, layout=abi.LAYOUT_PACKED))
    os_, ol = oracle.oracle_parse(g, abi.make_opts(0, 8, csum, ml))
    oracle.compare_exact(gp["summary"], gp["layers"], os_, ol)


@pytest.mark.gpu
def test_gpu_packed_layout_golden(engine):
    for path in golden_files():
        batch, variants = load_golden(path)
        for v, (opts, rsum, rlay) in variants.items():
            if not 0 < opts.max_layers <= abi.PACKED_MAX_LAYERS:
                opts = abi.make_opts(opts.parse_until_family, opts.parse_until_osi, bool(opts.want_checksums), 12)
            po = abi.make_opts(opts.parse_until_family, opts.parse_until_osi, bool(opts.want_checksums),
                               opts.max_layers, layout=abi.LAYOUT_PACKED)
            g = _device(engine, batch, po, tuples=False, stats=False)
            os_, ol = oracle.oracle_parse(batch, opts)
            oracle.compare_exact(g["summary"], g["layers"], os_, ol)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,ml,layout", [(2, 0, abi.LAYOUT_FIXED), (4, 0, abi.LAYOUT_FIXED), (4, 8, abi.LAYOUT_PACKED),
                                           (3, 8, abi.LAYOUT_FIXED), (5, 12, abi.LAYOUT_PACKED)])
def test_gpu_short_window(engine, cfg, ml, layout):
    """opts.window = PCPPX_WINDOW_SHORT (parse-only launches gather one 96-B round and no second one; stacks past it take
    the generic walk): summary, layers, tuples and collectStats identical to the default two-round window's and to the
    restatement's on configs 2-5 with checksums off (config 5's deep stacks run the generic walk), config 2 at its full
    1M through the bench's own output (tuples alone), a gapped batch, the host path, crafted stacks and every golden set
    under its option variants (checksum launches run their DEFAULT window under SHORT)."""
    from mutate import as_batch, crafted, crafted_l7

    from pcapplusplus_amd.engine import parse_on_device

    n = 1_000_000 if cfg == 2 else 100_000
    b = synth.config(cfg, n)
    short = abi.make_opts(0, 8, False, ml, abi.WINDOW_SHORT, layout)
    gs = _device(engine, b, short, summary=cfg != 2, stats=cfg != 2)
    if cfg == 2:  # bench config 2's launch: the 5-tuple extract alone
        _, _, ot = oracle.oracle_parse_tuples(b, short, threads=8)
        assert gs["tuples"].tobytes() == ot.tobytes()
        return
    gd = _device(engine, b, abi.make_opts(0, 8, False, ml, layout=layout))

    def lay(g):  # max_layers 0 writes no layers
        return g.get("layers", np.zeros((len(g["summary"]), 0), dtype=abi.LAYER_DTYPE))

    oracle.compare_exact(gs["summary"], lay(gs), gd["summary"], lay(gd))
    assert gs["tuples"].tobytes() == gd["tuples"].tobytes() and gs["proto_stats"] == gd["proto_stats"]
    sub = as_batch([b.packet(i) for i in range(0, n, 11)], gaps=True, seed=cfg)
    g = _device(engine, sub, short)
    os_, ol, ot = oracle.oracle_parse_tuples(sub, short, threads=8)
    assert g["tuples"].tobytes() == ot.tobytes()
    oracle.compare_exact(g["summary"], lay(g), os_, ol)
    if layout == abi.LAYOUT_FIXED and ml:
        h = engine.parse_host(b, short)  # the host path's chunked launches pick the same instance
        oracle.compare_exact(h[0], h[1], gs["summary"], gs["layers"])
    if cfg != 4 or ml:
        return
    cb = as_batch(crafted() + crafted_l7(), gaps=True, seed=29)
    for csum in (False, True):
        o = abi.make_opts(0, 8, csum, 16, abi.WINDOW_SHORT)
        s, lay = parse_on_device(engine, cb, o)
        os_, ol = oracle.oracle_parse(cb, o)
        oracle.compare_exact(s, lay, os_, ol)
    for path in golden_files():
        batch, variants = load_golden(path)
        for v, (opts, rsum, rlay) in variants.items():
            o = abi.make_opts(opts.parse_until_family, opts.parse_until_osi, bool(opts.want_checksums), opts.max_layers,
                              abi.WINDOW_SHORT)
            s, lay = parse_on_device(engine, batch, o)
            os_, ol = oracle.oracle_parse(batch, o)
            oracle.compare_exact(s, lay, os_, ol)


@pytest.mark.gpu
def test_gpu_summary_free_flow_launch(engine):
    """A flow table's launch (bench config 4): no summary, only the dense hash5 column and the collectStats counters
    (pcppx_records.summary = NULL) -- the keys equal the summary's hash5 of a full launch and the restatement's, the
    counters equal the full launch's, under the default and the SHORT window."""
    b = synth.config(4, 200_000)
    full = _device(engine, b, abi.make_opts(0, 8, False, 0), tuples=False, stats=True)
    for w in (abi.WINDOW_DEFAULT, abi.WINDOW_SHORT):
        g = _device(engine, b, abi.make_opts(0, 8, False, 0, w), summary=False, tuples=False, stats=True)
        assert "summary" not in g
        from pcapplusplus_amd.engine import parse_on_device_ex
        k = parse_on_device_ex(engine, b, abi.make_opts(0, 8, False, 0, w), summary=False, proto_stats=True,
                               flow_keys=True)
        assert (k["flow_keys"] == full["summary"]["hash5"]).all()
        assert k["proto_stats"] == full["proto_stats"] == g["proto_stats"]
    idx = np.arange(0, b.n, 17)
    from mutate import as_batch
    sub = as_batch([b.packet(int(i)) for i in idx])
    os_, _ = oracle.oracle_parse(sub, abi.make_opts(0, 8, False, 0))
    assert (k["flow_keys"][idx] == os_["hash5"]).all()
