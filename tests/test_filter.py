"""DpdkExample-FilterTraffic's worker (AppWorkerThread.h:85-139) on the engine's records.

CPU: the Python restatement of the worker (oracle.oracle_filter over the restatement's records) equals
the reference worker loop built from source (real PacketMatchingEngine.h + hash5Tuple flow table +
collectStats, oracle/ref_harness.cpp: pcppx_ref_filter) for packets the engine finishes on the device.
GPU: pcppx_filter_device equals both, across batch boundaries (seq_base) with a persistent flow table.
The L7 counters (HTTP/DNS/SSL) are the device's for every packet it settles (the first L7 layer of a
NEEDS_HOST_L7 packet is classified on the device); the batches compared with the reference hold the
settled packets, and the unsettled rest is counted in needs_host_count (checked against the restatement).
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from conftest import golden_files, load_golden
from pcapplusplus_amd import abi, synth

L7_STATS = ("needs_host_count",)
OPTS = abi.make_opts(0, 8, False, 16)


def device_finishable(batch):
    """Packets whose counters the device settles (oracle.stats_settled, the filter kernel's rule): no
    NEEDS_HOST_PROTO / bad records, and no L7 payload that tunnels a further packet (VXLAN, GTPv1)."""
    s, lay = oracle.oracle_parse(batch, OPTS)
    ok, _ = oracle.stats_settled(batch, s, lay)
    keep = np.nonzero(ok)[0]
    return batch.take(keep) if hasattr(batch, "take") else _take(batch, keep)


def _take(batch, idx):
    from pcapplusplus_amd.pcap import from_packets

    return from_packets([batch.packet(int(i)) for i in idx], batch.linktype)


def specs_for(batch, seed: int):
    """Match specs drawn from the batch itself so that matches exist: an IPv4 source address, a port of
    a TCP/UDP layer, each protocol, combinations, and the match-everything spec."""
    s, lay = oracle.oracle_parse(batch, OPTS)
    rng = np.random.default_rng(seed)
    v4 = [(i, int(lay[i, k]["offset"])) for i in range(batch.n) for k in range(min(int(s["n_layers"][i]), 16))
          if lay[i, k]["proto"] == 2][:5000]
    l4 = [(i, int(lay[i, k]["offset"])) for i in range(batch.n) for k in range(min(int(s["n_layers"][i]), 16))
          if lay[i, k]["proto"] in (4, 5)][:5000]
    out = [oracle.make_spec(), oracle.make_spec(protocol=4), oracle.make_spec(protocol=5)]
    for _ in range(2):
        if v4:
            i, o = v4[rng.integers(len(v4))]
            pkt = batch.packet(i)
            out.append(oracle.make_spec(src_ip=int.from_bytes(pkt[o + 12:o + 16], "little")))
            out.append(oracle.make_spec(dst_ip=int.from_bytes(pkt[o + 16:o + 20], "little"), protocol=4))
        if l4:
            i, o = l4[rng.integers(len(l4))]
            pkt = batch.packet(i)
            out.append(oracle.make_spec(dst_port=pkt[o + 2] << 8 | pkt[o + 3]))
            out.append(oracle.make_spec(src_port=pkt[o] << 8 | pkt[o + 1], protocol=5))
    return out


def batches():
    out = [(p.stem, load_golden(p)[0]) for p in golden_files()
           if p.stem in ("pcap_lt1", "synth_cfg3", "synth_cfg4", "dat_ethernet")]
    out.append(("flows", synth.imix(20000, 77, flows=300, corrupt_frac=0.0)))
    return out


def compare_stats(got: dict, want: dict):
    for k in abi.STATS_FIELDS:
        if k in L7_STATS:
            continue
        assert got[k] == want[k], (k, got[k], want[k])


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build absent")
@pytest.mark.parametrize("name,batch", batches(), ids=lambda x: x if isinstance(x, str) else "")
def test_oracle_filter_matches_reference_worker(name, batch):
    b = device_finishable(batch)
    s, lay = oracle.oracle_parse(b, OPTS)
    for k, spec in enumerate(specs_for(b, 1)):
        om, ost = oracle.oracle_filter(b, s, lay, spec)
        rm, rst = oracle.ref_filter(b, spec)
        mism = np.nonzero(om != rm)[0]
        assert len(mism) == 0, (name, k, mism[:10])
        compare_stats(ost, rst)


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build absent")
def test_flow_table_persists_across_batches():
    b = device_finishable(batches()[-1][1])
    spec = specs_for(b, 3)[3]
    s, lay = oracle.oracle_parse(b, OPTS)
    rm, rst = oracle.ref_filter(b, spec)
    half = b.n // 2
    ft = {}
    m0, st0 = oracle.oracle_filter(b.slice(0, half), s[:half], lay[:half], spec, ft)
    m1, st1 = oracle.oracle_filter(b.slice(half, b.n), s[half:], lay[half:], spec, ft)
    assert np.array_equal(np.concatenate([m0, m1]), rm)
    compare_stats({k: st0[k] + st1[k] for k in st0}, rst)


# ---------------------------------------------------------------- device
def gpu_filter(engine, batch, spec, splits=(), capacity=1 << 16, max_layers=16):
    """Parse + filter a host batch on cuda:0 in consecutive sub-batches (a persistent flow table)."""
    import torch

    from pcapplusplus_amd.engine import to_device

    dev = "cuda:0"
    keys = torch.zeros(capacity, dtype=torch.int64, device=dev)
    first = torch.zeros(capacity, dtype=torch.int64, device=dev)
    stats = torch.zeros(len(abi.STATS_FIELDS), dtype=torch.int64, device=dev)
    matched = []
    bounds = [0, *splits, batch.n]
    opts = abi.make_opts(0, 8, False, max_layers)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for a, z in zip(bounds[:-1], bounds[1:]):
        sub = batch.slice(a, z)
        n = sub.n
        data, offsets, caplens = to_device(sub, dev)
        summary = torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device=dev)
        layers = torch.zeros(max(n * max_layers, 1) * 8, dtype=torch.uint8, device=dev)
        m = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
        engine.parse_device(data, offsets, caplens, n, sub.linktype, opts, summary, layers, stream)
        engine.filter_device(data, offsets, caplens, n, sub.linktype, summary, layers, max_layers, spec, a,
                             keys, first, capacity, m, stats, stream)
        torch.cuda.synchronize(dev)
        matched.append(m.cpu().numpy()[:n])
    st = stats.cpu().numpy().view(np.uint64)
    return np.concatenate(matched), {k: int(v) for k, v in zip(abi.STATS_FIELDS, st)}


@pytest.mark.gpu
@pytest.mark.parametrize("name,batch", batches(), ids=lambda x: x if isinstance(x, str) else "")
def test_gpu_filter(engine, name, batch):
    b = device_finishable(batch)
    s, lay = oracle.oracle_parse(b, OPTS)
    for k, spec in enumerate(specs_for(b, 1)):
        gm, gst = gpu_filter(engine, b, spec, splits=(b.n // 3, b.n // 2))
        om, ost = oracle.oracle_filter(b, s, lay, spec)
        mism = np.nonzero(gm != om)[0]
        assert len(mism) == 0, (name, k, mism[:10])
        compare_stats(gst, ost)
        assert gst["needs_host_count"] == ost["needs_host_count"] == 0
        if oracle.ref_available():
            rm, rst = oracle.ref_filter(b, spec)
            assert np.array_equal(gm, rm)
            compare_stats(gst, rst)


@pytest.mark.gpu
def test_gpu_filter_large_vs_reference(engine):
    """200k-packet flow workload in 4 sub-batches against the reference worker (or the restatement)."""
    b = synth.imix(200_000, 91, flows=5000, corrupt_frac=0.0)
    for spec in specs_for(b.slice(0, 20000), 5)[:6]:
        gm, gst = gpu_filter(engine, b, spec, splits=(50_000, 100_000, 150_000), capacity=1 << 14)
        if oracle.ref_available():
            rm, rst = oracle.ref_filter(b, spec)
        else:
            s, lay = oracle.oracle_parse(b, OPTS, threads=8)
            rm, rst = oracle.oracle_filter(b, s, lay, spec)
        assert np.array_equal(gm, rm)
        compare_stats(gst, rst)


@pytest.mark.gpu
def test_gpu_filter_rejects_bad_args(engine):
    import torch

    dev = "cuda:0"
    t = torch.zeros(64, dtype=torch.int64, device=dev)
    spec = oracle.make_spec()
    with pytest.raises(RuntimeError):  # capacity not a power of two
        engine.filter_device(t, t, t, 4, 1, t, t, 8, spec, 0, t, t, 6, t, t)
    with pytest.raises(RuntimeError):  # max_layers 0: no layer records to read addresses from
        engine.filter_device(t, t, t, 4, 1, t, t, 0, spec, 0, t, t, 8, t, t)


@pytest.mark.gpu
@pytest.mark.parametrize("name,batch", batches(), ids=lambda x: x if isinstance(x, str) else "")
def test_gpu_filter_host(engine, name, batch):
    """pcppx_filter_batch_host: the context-held flow table across two calls, stats cumulative."""
    b = device_finishable(batch)
    s, lay = oracle.oracle_parse(b, OPTS)
    for spec in specs_for(b, 2)[:5]:
        engine.filter_reset(1 << 12)
        half = b.n // 2
        m0, _ = engine.filter_host(b.slice(0, half), spec)
        m1, gst = engine.filter_host(b.slice(half, b.n), spec)
        om, ost = oracle.oracle_filter(b, s, lay, spec)
        assert np.array_equal(np.concatenate([m0, m1]), om)
        compare_stats(gst, ost)


@pytest.mark.gpu
def test_gpu_filter_host_multichunk(engine):
    """A batch larger than one host-path chunk (256K packets): chunks share the flow table in order."""
    b = synth.imix(600_000, 17, flows=20_000, corrupt_frac=0.0)
    spec = specs_for(b.slice(0, 20000), 9)[5]
    engine.filter_reset(0)
    gm, gst = engine.filter_host(b, spec)
    if oracle.ref_available():
        rm, rst = oracle.ref_filter(b, spec)
    else:
        s, lay = oracle.oracle_parse(b, OPTS, threads=8)
        rm, rst = oracle.oracle_filter(b, s, lay, spec)
    assert np.array_equal(gm, rm)
    compare_stats(gst, rst)


def test_l7_counters_cover_every_class():
    """The settled fixture packets exercise HTTP requests and responses, DNS and SSL."""
    b = device_finishable([x for n, x in batches() if n == "pcap_lt1"][0])
    s, lay = oracle.oracle_parse(b, OPTS)
    settled, l7 = oracle.stats_settled(b, s, lay)
    assert settled.all()
    for bit in (1, 2, 4):
        assert ((l7 & bit) != 0).sum() > 50, bit
    http_resp = [i for i in np.nonzero(l7 & 1)[0] if b.packet(int(i))[int(lay[i, int(s["l4_layer"][i])]["offset"])
                                                                        :][:2] == b"\x00\x50"]
    assert http_resp, "no HTTP response among the fixtures"
    # with no parse-until family the parse builds those layers itself: HTTPRequest / HTTPResponse, SSL, DNS
    for proto in (6, 7, 13, 18):
        assert (lay["proto"] == proto).any(), proto


@pytest.mark.gpu
def test_gpu_filter_mixed_settled_and_host(engine):
    """Unsettled packets (out-of-scope L2/L3 layers, tunnels) are counted in needs_host_count and their
    L7 counters left out, exactly as the restatement decides."""
    b = [x for n, x in batches() if n == "pcap_lt1"][0]
    s, lay = oracle.oracle_parse(b, OPTS)
    spec = oracle.make_spec()
    gm, gst = gpu_filter(engine, b, spec, splits=(b.n // 2,))
    om, ost = oracle.oracle_filter(b, s, lay, spec)
    assert np.array_equal(gm, om)
    for k in abi.STATS_FIELDS:
        assert gst[k] == ost[k], (k, gst[k], ost[k])
    assert ost["needs_host_count"] > 0


@pytest.mark.gpu
def test_gpu_filter_table_full_is_counted(engine):
    """A flow table too small for the matched flows cannot hold the reference's unordered_map: the packets whose
    flow finds no free slot are counted in flow_table_full (pcppx.h), and with room to spare the count is 0."""
    b = device_finishable([x for n, x in batches() if n == "pcap_lt1"][0])
    spec = oracle.make_spec()
    s, lay = oracle.oracle_parse(b, OPTS)
    _, ost = oracle.oracle_filter(b, s, lay, spec)
    _, big = gpu_filter(engine, b, spec)
    assert big["flow_table_full"] == 0 and big["matched_packets"] == ost["matched_packets"]
    _, small = gpu_filter(engine, b, spec, capacity=8)
    flows = ost["matched_tcp_flows"] + ost["matched_udp_flows"]
    assert flows > 8
    assert 0 < small["flow_table_full"] <= ost["matched_packets"]
