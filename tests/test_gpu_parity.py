"""HIP engine parity on an MI355X, through the C ABI (libpcppx.so).

Bar: bit-exact. Every record field of the device path equals the C restatement (oracle/) on every
packet, and equals the reference Packet++'s golden records under the engine contract (unflagged packets
fully, flagged packets as an exact layer prefix). Full-size batches are checked through size-independent
properties plus a record-for-record restatement comparison of every packet.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from conftest import golden_files, load_golden
from mutate import as_batch, crafted, crafted_http, crafted_l7, mutate
from pcapplusplus_amd import abi, synth
from pcapplusplus_amd.engine import parse_on_device
from pcapplusplus_amd.pcap import from_packets

pytestmark = pytest.mark.gpu


def run(engine, batch, opts, kernel: int):
    """kernel 0: the product path (libpcppx.so); 1: the lane-per-packet cross-check kernel of the tools-only
    A/B library (tools/ab/libpcppx_ab.so), an independent implementation of the same records."""
    if kernel == 0:
        return parse_on_device(engine, batch, opts)
    from tools import ab

    return ab.parse_on_device(batch, opts, ab.LANE)


@pytest.mark.parametrize("kernel", [0, 1], ids=["tile", "lane"])
@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.stem)
def test_gpu_golden(engine, path, kernel):
    batch, variants = load_golden(path)
    for v, (opts, rsum, rlay) in variants.items():
        gsum, glay = run(engine, batch, opts, kernel)
        osum, olay = oracle.oracle_parse(batch, opts)
        oracle.compare_exact(gsum, glay, osum, olay)
        oracle.compare_engine_to_reference(gsum, glay, rsum, rlay)


@pytest.mark.parametrize("kernel", [0, 1], ids=["tile", "lane"])
@pytest.mark.parametrize("gaps", [False, True])
def test_gpu_crafted_deep_stacks(engine, gaps, kernel):
    b = as_batch(crafted(), gaps=gaps, seed=11)
    for opts in (abi.make_opts(), abi.make_opts(4, 8, True, 16), abi.make_opts(0, 3, True, 5),
                 abi.make_opts(0, 8, True, 0), abi.make_opts(0, 8, False, 16),
                 abi.make_opts(0, 8, True, 16, abi.WINDOW_DEEP), abi.make_opts(4, 8, True, 16, abi.WINDOW_DEEP)):
        g = run(engine, b, opts, kernel)
        o = oracle.oracle_parse(b, opts)
        oracle.compare_exact(g[0], g[1], o[0], o[1])
        if oracle.ref_available():
            r = oracle.ref_parse(b, opts)
            oracle.compare_engine_to_reference(g[0], g[1], r[0], r[1])


@pytest.mark.gpu
@pytest.mark.parametrize("gaps", [False, True])
def test_gpu_http_text_walks(engine, gaps):
    """HTTP first lines and header fields ending at every offset of the text-walk groups and far past the LDS window
    (mutate.crafted_http), through the checksum instance (2-dword groups) and the parse-only ones (4-dword groups, with
    and without the second gather round): every record equal to the restatement's and the reference Packet++'s."""
    b = as_batch(crafted_http(), gaps=gaps, seed=31)
    for opts in (abi.make_opts(0, 8, True, 16), abi.make_opts(0, 8, False, 16),
                 abi.make_opts(0, 8, False, 16, abi.WINDOW_SHORT), abi.make_opts(0, 8, True, 16, abi.WINDOW_DEEP),
                 abi.make_opts(0x607, 8, False, 16), abi.make_opts(0, 7, False, 16)):
        g = run(engine, b, opts, 0)
        o = oracle.oracle_parse(b, opts)
        oracle.compare_exact(g[0], g[1], o[0], o[1])
        if oracle.ref_available():
            r = oracle.ref_parse(b, opts)
            oracle.compare_engine_to_reference(g[0], g[1], r[0], r[1])


@pytest.mark.parametrize("kernel", [0, 1], ids=["tile", "lane"])
@pytest.mark.parametrize("gaps", [False, True])
def test_gpu_crafted_l7_payloads(engine, gaps, kernel):
    """The L7 content checks (HTTP request / response first line, SSL record header, DNS lengths) at their edges,
    on the fast path (Eth/IPv4) and the generic walk (VLAN/IPv6), payload bytes in and past the LDS window."""
    b = as_batch(crafted_l7(), gaps=gaps, seed=17)
    # parse-until variants around the built HTTP / SSL / DNS layers: TCP, HTTP (request|response), SSL, DNS and
    # UDP families, OSI 4 / 6 / 7
    for opts in (abi.make_opts(), abi.make_opts(4, 8, True, 16), abi.make_opts(0, 4, True, 16),
                 abi.make_opts(0, 8, False, 0), abi.make_opts(0x607, 8, True, 16), abi.make_opts(18, 8, True, 16),
                 abi.make_opts(13, 8, True, 16), abi.make_opts(5, 8, True, 16), abi.make_opts(0, 6, True, 16),
                 abi.make_opts(0, 7, True, 8)):
        g = run(engine, b, opts, kernel)
        o = oracle.oracle_parse(b, opts)
        oracle.compare_exact(g[0], g[1], o[0], o[1])
        if oracle.ref_available() and opts.max_layers:
            r = oracle.ref_parse(b, opts)
            oracle.compare_engine_to_reference(g[0], g[1], r[0], r[1])
            oracle.check_flag_contract(g[0], r[0], r[1], b)


@pytest.mark.parametrize("kernel", [0, 1], ids=["tile", "lane"])
@pytest.mark.parametrize("gaps", [False, True])
def test_gpu_mutations(engine, gaps, kernel):
    seedb, _ = load_golden([p for p in golden_files() if p.stem == "pcap_lt1"][0])
    pk = [seedb.packet(i) for i in range(seedb.n)]
    b = as_batch(mutate(pk, 40000, 5), gaps=gaps, seed=5)
    g = run(engine, b, abi.make_opts(), kernel)
    o = oracle.oracle_parse(b, threads=8)
    oracle.compare_exact(g[0], g[1], o[0], o[1])


@pytest.mark.parametrize("kernel", [0, 1], ids=["tile", "lane"])
@pytest.mark.parametrize("order", ["tile-local", "global"])
def test_gpu_permuted_descriptors(engine, order, kernel):
    """Descriptors out of address order: permuted inside each 64-packet tile (the span stream reads a
    tile's bytes in a different order than its packets) and across the whole batch (spans too sparse to
    stream: whole-chunk sums straight from HBM). Records must not change."""
    b = synth.config(3, 100_000)
    rng = np.random.default_rng(9)
    n = b.n
    if order == "global":
        perm = rng.permutation(n)
    else:
        perm = np.concatenate([t0 + rng.permutation(min(64, n - t0)) for t0 in range(0, n, 64)])
    pb = type(b)(b.data, b.offsets[perm].copy(), b.caplens[perm].copy(), b.linktype)
    opts = abi.make_opts(0, 8, True, 8)
    g = run(engine, pb, opts, kernel)
    o = oracle.oracle_parse(pb, abi.make_opts(0, 8, True, 8), threads=8)
    oracle.compare_exact(g[0], g[1], o[0], o[1])


@pytest.mark.parametrize("kernel", [0, 1], ids=["tile", "lane"])
@pytest.mark.parametrize("linktype", [0, 113, 276, 104, 239])
def test_gpu_link_layers(engine, linktype, kernel):
    """Linux SLL / SLL2 / Null-Loopback / Cisco HDLC / NFLOG first layers (Packet::createFirstLayer, Packet.cpp:827-923) on the generic
    walk: crafted edge cases (lengths 0-23, every dispatch value and family encoding) and their mutations, packed
    and with gaps, equal to the restatement (itself pinned to the reference in test_oracle_fuzz)."""
    from mutate import crafted_linklayers

    seeds = crafted_linklayers()[linktype]
    pk = seeds + mutate(seeds, 3000, linktype + 1)
    for gaps in (False, True):
        b = as_batch(pk, gaps=gaps, seed=linktype)
        b.linktype = linktype
        for opts in (abi.make_opts(), abi.make_opts(4, 8, True, 16), abi.make_opts(0, 2, True, 16),
                     abi.make_opts(0, 8, False, 3)):
            g = run(engine, b, opts, kernel)
            o = oracle.oracle_parse(b, opts)
            oracle.compare_exact(g[0], g[1], o[0], o[1])


def test_gpu_edge_descriptors(engine):
    pk = [b"", b"\x01", bytes(13), bytes(14), bytes(70000), bytes(60)]
    b = from_packets(pk)
    b.caplens[5] = 1 << 20  # beyond data_len
    g = parse_on_device(engine, b)
    o = oracle.oracle_parse(b)
    oracle.compare_exact(g[0], g[1], o[0], o[1])
    assert g[0]["flags"][4] == abi.F_OVERSIZE and g[0]["flags"][5] == abi.F_BAD_DESC


@pytest.mark.parametrize("cfg,n", [(1, 10_000), (2, 1_000_000), (3, 200_000), (4, 200_000), (5, 200_000)])
def test_gpu_synthetic_configs(engine, cfg, n):
    b = synth.config(cfg, n)
    for opts in (abi.make_opts(), abi.make_opts(0, 8, False, 8)):
        g = parse_on_device(engine, b, opts)
        o = oracle.oracle_parse(b, opts, threads=8)
        oracle.compare_exact(g[0], g[1], o[0], o[1])
        assert not (g[0]["flags"] & abi.F_NEEDS_HOST).any()


@pytest.mark.parametrize("size", [64, 512, 1500])
def test_gpu_sized_batches(engine, size):
    """bench.py --sizes 64|512|1500: config 3's batch at one packet size (the per-size lines), checksums on, the
    summary + PACKED rows as the bench writes them, and FIXED rows; every record equal to the restatement's."""
    b = synth.imix(200_000, 3, sizes=(size,), weights=(1,))
    for layout in (abi.LAYOUT_PACKED, abi.LAYOUT_FIXED):
        opts = abi.make_opts(0, 8, True, 8, layout=layout)
        g = parse_on_device(engine, b, opts)
        o = oracle.oracle_parse(b, abi.make_opts(0, 8, True, 8), threads=8)
        lay = abi.unpack_layers(g[0], g[1], 8) if layout == abi.LAYOUT_PACKED else g[1]
        oracle.compare_exact(g[0], lay, o[0], o[1])
        assert not (g[0]["flags"] & abi.F_NEEDS_HOST).any()


def test_gpu_host_path_matches_device_path(engine):
    """pcppx_parse_batch_host (chunked, three slots) equals the device path: packed pageable input
    (staged by the copy threads), pinned input (DMA straight from the caller's bytes), pinned input and
    pinned record arrays (records DMA'd straight into them, no drain copy), and a gapped batch (per-packet
    gather)."""
    from pcapplusplus_amd.engine import pinned_copy, pinned_records

    b = synth.config(3, 600_000)
    opts = abi.make_opts(0, 8, True, 8)
    d = parse_on_device(engine, b, opts)
    h = engine.parse_host(b, opts)
    oracle.compare_exact(h[0], h[1], d[0], d[1])
    pb, buf = pinned_copy(b)
    hp = engine.parse_host(pb, opts)
    oracle.compare_exact(hp[0], hp[1], d[0], d[1])
    out, keep = pinned_records(b.n, opts.max_layers)
    hpo = engine.parse_host(pb, opts, out)
    oracle.compare_exact(hpo[0], hpo[1], d[0], d[1])
    del hpo, out
    for k in keep:
        k.free()
    buf.free()
    g = as_batch([b.packet(i) for i in range(20_000)], gaps=True, seed=3)
    hg = engine.parse_host(g, opts)
    dg = parse_on_device(engine, g, opts)
    oracle.compare_exact(hg[0], hg[1], dg[0], dg[1])


def test_gpu_full_size_imix_properties(engine):
    """Config 3 at its full 10M size: properties that hold independently of size, and every record of every packet
    bit-exact against the multi-threaded restatement (round 4: all 10M, no sample); the bench's own launch (PACKED +
    brief) equal to it on every packet."""
    n = 10_000_000
    b = synth.config(3, n)
    opts = abi.make_opts(0, 8, True, 8)
    s, lay = parse_on_device(engine, b, opts)
    fl = s["flags"]
    assert not (fl & abi.F_NEEDS_HOST).any()
    # every packet: Eth [VLAN] IP L4 Payload, no trailer (synthetic lengths are exact)
    assert ((s["n_layers"] >= 4) & (s["n_layers"] <= 5)).all()  # Eth [VLAN] IP L4 Payload
    assert not (fl & abi.F_TRAILER).any()
    # checksum verdicts: exactly the corrupted packets fail
    bad = int(((fl & abi.F_L4_CSUM) != 0).sum() - ((fl & abi.F_L4_CSUM_OK) != 0).sum()) + \
        int(((fl & abi.F_IP_CSUM) != 0).sum() - ((fl & abi.F_IP_CSUM_OK) != 0).sum())
    assert bad == b.meta["corrupted"]
    # last layer ends at caplen
    last = lay[np.arange(n), s["n_layers"] - 1]
    assert (last["offset"].astype(np.int64) + last["data_len"] == b.caplens).all()
    # every packet bit-exact against the restatement
    o = oracle.oracle_parse(b, opts, threads=16)
    oracle.compare_exact(s, lay, o[0], o[1])
    _bench_launch_equals(engine, b, opts, s, lay)


def _bench_launch_equals(engine, b, opts, s, lay):
    """bench.py's own timed launch at full size -- PACKED rows + the 16-B brief, no summary (configs 3 / 5) -- decodes
    to the FIXED parse's rows and briefs on every packet (round-4 verdict: the full-size comparison ran FIXED only)."""
    from pcapplusplus_amd.engine import parse_on_device_ex

    po = abi.make_opts(opts.parse_until_family, opts.parse_until_osi, bool(opts.want_checksums), opts.max_layers,
                       layout=abi.LAYOUT_PACKED)
    g = parse_on_device_ex(engine, b, po, summary=False, brief=True)
    half = s.view(np.uint8).reshape(len(s), 32)[:, :16].copy().view(abi.BRIEF_DTYPE).ravel()
    assert g["brief"].tobytes() == half.tobytes()
    nl = np.minimum(s["n_layers"], opts.max_layers)
    valid = np.arange(opts.max_layers)[None, :] < nl[:, None]
    zero = np.zeros(1, abi.LAYER_DTYPE)
    assert np.where(valid, g["layers"], zero).tobytes() == np.where(valid, lay, zero).tobytes()


def test_gpu_full_size_deep_encap_properties(engine):
    """Config 5 at its full 10M size: every stack is parsed to its Payload with no host fallback, the
    layer chain is contiguous (each layer starts at its predecessor's offset + header length) and the last
    layer ends at caplen; and every record of every packet bit-exact against the multi-threaded restatement."""
    n = 10_000_000
    b = synth.config(5, n)
    opts = abi.make_opts(0, 8, False, 12)
    s, lay = parse_on_device(engine, b, opts)
    fl = s["flags"]
    assert not (fl & (abi.F_NEEDS_HOST | abi.F_DEPTH_OVERFLOW | abi.F_TRAILER)).any()
    nl = s["n_layers"].astype(np.int64)
    assert ((nl >= 3) & (nl <= 10)).all()
    rows = np.arange(n)
    last = lay[rows, nl - 1]
    assert (last["proto"] == 25).all()  # GenericPayload
    assert (last["offset"].astype(np.int64) + last["data_len"] == b.caplens).all()
    for k in range(1, 10):
        m = nl > k
        prev, cur = lay[m, k - 1], lay[m, k]
        assert (prev["offset"].astype(np.int64) + prev["hdr_len"] == cur["offset"]).all(), k
    o = oracle.oracle_parse(b, opts, threads=16)
    oracle.compare_exact(s, lay, o[0], o[1])
    _bench_launch_equals(engine, b, opts, s, lay)


def test_gpu_flow_hash_symmetry_and_flow_table(engine):
    """Config 4 shape: both directions of a flow share hash5Tuple; the device flow table's per-flow
    counters equal a host group-by over the same hashes (FilterTraffic's flow table)."""
    import torch

    b = synth.config(4, 500_000)
    opts = abi.make_opts(0, 8, False, 0)
    s, _ = parse_on_device(engine, b, opts)
    fid = b.meta["flow_id"]
    order = np.argsort(fid, kind="stable")
    f_sorted, h_sorted = fid[order], s["hash5"][order]
    same_flow = f_sorted[1:] == f_sorted[:-1]
    assert (h_sorted[1:][same_flow] == h_sorted[:-1][same_flow]).all()
    # device flow table
    dev = "cuda:0"
    summ = torch.from_numpy(s.view(np.uint8).copy()).to(dev)
    caps = torch.from_numpy(b.caplens.view(np.int32)).to(dev)
    cap = 1 << 21
    keys = torch.zeros(cap, dtype=torch.int32, device=dev)
    pk = torch.zeros(cap, dtype=torch.int64, device=dev)
    by = torch.zeros(cap, dtype=torch.int64, device=dev)
    st = torch.zeros(4, dtype=torch.int64, device=dev)
    engine.flow_count_device(summ, caps, b.n, keys, pk, by, cap, st, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    k = keys.cpu().numpy().view(np.uint32)
    used = k != 0
    got = dict(zip(k[used].tolist(), zip(pk.cpu().numpy()[used].tolist(), by.cpu().numpy()[used].tolist())))
    uniq, inv = np.unique(s["hash5"], return_inverse=True)
    cnt = np.bincount(inv)
    byt = np.bincount(inv, weights=b.caplens.astype(np.float64)).astype(np.int64)
    want = {int(u): (int(c), int(y)) for u, c, y in zip(uniq, cnt, byt) if u != 0}
    assert got == want
    assert st.cpu().numpy()[2] == 0


def _device_flow_table(engine, s, caplens, n, cap, calls=1):
    import torch

    dev = "cuda:0"
    summ = torch.from_numpy(s.view(np.uint8).copy()).to(dev)
    caps = torch.from_numpy(caplens.view(np.int32)).to(dev)
    keys = torch.zeros(cap, dtype=torch.int32, device=dev)
    pk = torch.zeros(cap, dtype=torch.int64, device=dev)
    by = torch.zeros(cap, dtype=torch.int64, device=dev)
    st = torch.zeros(4, dtype=torch.int64, device=dev)
    for _ in range(calls):
        engine.flow_count_device(summ, caps, n, keys, pk, by, cap, st, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    k = keys.cpu().numpy().view(np.uint32)
    used = k != 0
    got = dict(zip(k[used].tolist(), zip(pk.cpu().numpy()[used].tolist(), by.cpu().numpy()[used].tolist())))
    return got, st.cpu().numpy()


def _host_group_by(s, caplens, scale=1):
    uniq, inv = np.unique(s["hash5"], return_inverse=True)
    cnt = np.bincount(inv)
    byt = np.bincount(inv, weights=caplens.astype(np.float64)).astype(np.int64)
    return {int(u): (int(c) * scale, int(y) * scale) for u, c, y in zip(uniq, cnt, byt)}


def test_gpu_flow_table_multi_batch_blocks_and_repeated_calls(engine):
    """2M Zipf packets: every persistent block aggregates several LDS batches (hot flows kept in LDS
    between them) and two calls accumulate into the same table; the counters equal twice a host
    group-by, flow key 0 (no 5-tuple) goes to the stats counters, nothing is lost."""
    b = synth.imix(2_000_000, 7, corrupt_frac=0.0, flows=200_000)
    s, _ = parse_on_device(engine, b, abi.make_opts(0, 8, False, 0))
    got, st = _device_flow_table(engine, s, b.caplens, b.n, 1 << 20, calls=2)
    want = _host_group_by(s, b.caplens, scale=2)
    zero = want.pop(0, (0, 0))
    assert got == want
    assert (int(st[0]), int(st[1]), int(st[2])) == (zero[0], zero[1], 0)


def test_gpu_flow_table_many_batches_per_block(engine):
    """9M packets with Zipf(1.1) flow keys over 1M flows (a synthetic summary: only hash5 and caplen are read):
    each of the 256 persistent blocks aggregates 8-9 LDS batches of 4096 packets, so hot flows stay in LDS across
    many flushes and cold keys ahead of them in their probe chains are cleared between batches. Per-flow counters
    equal a host group-by exactly; key 0 goes to the stats counters."""
    n = 9_000_000
    rng = np.random.default_rng(5)
    ranks = np.minimum(rng.zipf(1.1, n), 1_000_000).astype(np.uint64)
    keys = ((ranks * 0x9E3779B1) & 0xFFFFFFFF).astype(np.uint32)  # distinct per rank, hot ranks first
    keys[rng.random(n) < 0.001] = 0
    s = np.zeros(n, dtype=abi.SUMMARY_DTYPE)
    s["hash5"] = keys
    caplens = rng.integers(60, 1515, n).astype(np.uint32)
    got, st = _device_flow_table(engine, s, caplens, n, 1 << 21)
    want = _host_group_by(s, caplens)
    zero = want.pop(0, (0, 0))
    assert len(want) > 100_000 and max(c for c, _ in want.values()) > n // 20
    assert got == want
    assert (int(st[0]), int(st[1]), int(st[2])) == (zero[0], zero[1], 0)


def test_gpu_flow_keys_column(engine):
    """pcppx_records.flow_keys: the parse writes every packet's hash5 into the dense column (device and host paths), and
    pcppx_flow_count_keys_device over it builds exactly the table pcppx_flow_count_device builds from the summaries."""
    import torch

    from pcapplusplus_amd.engine import to_device

    b = synth.imix(1_500_000, 9, corrupt_frac=0.0, flows=100_000)
    dev = "cuda:0"
    data, offs, caps = to_device(b, dev)
    n = b.n
    summ = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    fk = torch.full((n,), -1, dtype=torch.int32, device=dev)
    st0 = torch.cuda.current_stream().cuda_stream
    for csum in (False, True):
        engine.parse_device(data, offs, caps, n, b.linktype, abi.make_opts(0, 8, csum, 0), summ, None, st0, fk)
        torch.cuda.synchronize()
        s = summ.cpu().numpy().view(abi.SUMMARY_DTYPE)
        assert np.array_equal(fk.cpu().numpy().view(np.uint32), s["hash5"])
    cap = 1 << 18
    tabs = []
    for dense in (False, True):
        keys = torch.zeros(cap, dtype=torch.int32, device=dev)
        pk = torch.zeros(cap, dtype=torch.int64, device=dev)
        by = torch.zeros(cap, dtype=torch.int64, device=dev)
        stt = torch.zeros(4, dtype=torch.int64, device=dev)
        for _ in range(2):
            if dense:
                engine.flow_count_keys_device(fk, caps, n, keys, pk, by, cap, stt, st0)
            else:
                engine.flow_count_device(summ, caps, n, keys, pk, by, cap, stt, st0)
        torch.cuda.synchronize()
        k = keys.cpu().numpy().view(np.uint32)
        used = k != 0  # slot positions depend on the claim order: compare by key
        tabs.append((dict(zip(k[used].tolist(), zip(pk.cpu().numpy()[used].tolist(), by.cpu().numpy()[used].tolist()))),
                     stt.cpu().numpy().tolist()))
    assert tabs[0] == tabs[1] and len(tabs[0][0]) > 50_000
    sub = b.slice(0, 200_000)
    opts = abi.make_opts(0, 8, True, 0)
    out = (np.zeros(sub.n, dtype=abi.SUMMARY_DTYPE), np.zeros(1, dtype=abi.LAYER_DTYPE))
    hk = np.zeros(sub.n, dtype=np.uint32)
    rec = abi.Records(out[0].ctypes.data, None, hk.ctypes.data)
    bb = sub.c_batch()
    import ctypes as C
    abi.check(engine.lib.pcppx_parse_batch_host(engine.ctx, C.byref(bb), C.byref(opts), C.byref(rec)), "host")
    assert np.array_equal(hk, out[0]["hash5"]) and hk.any()


@pytest.mark.parametrize("cap", [256, 1024, 1 << 14, 1 << 16])
def test_gpu_flow_table_small_capacity_loses_nothing(engine, cap):
    """A small table with far fewer flows than slots (a fifth of capacity) loses no flow: every region of the
    partitioned table keeps at least 4096 slots (a table of up to 4096 slots is one region), so a flow only fails
    when its region is full, as in the reference's never-full unordered_map (AppWorkerThread.h:99-125). Per-flow
    counters exact, stats[2] == 0, over 300k packets in several calls."""
    rng = np.random.default_rng(cap)
    n, flows = 300_000, cap // 5
    pool = rng.choice(np.arange(1, 1 << 32, dtype=np.uint64), size=flows, replace=False).astype(np.uint32)
    s = np.zeros(n, dtype=abi.SUMMARY_DTYPE)
    s["hash5"] = pool[rng.integers(0, flows, n)]
    caplens = rng.integers(60, 1515, n).astype(np.uint32)
    got, st = _device_flow_table(engine, s, caplens, n, cap, calls=2)
    want = _host_group_by(s, caplens, scale=2)
    assert int(st[2]) == 0
    assert got == want


@pytest.mark.gpu
def test_gpu_flow_table_partition_queue_overflow_exact(engine):
    """Keys crafted so that every one falls in one partition of the table (flow_part: the top 9 bits of
    key * 0x9E3779B1), distinct per packet: the partition's record queue (1.25 x the even share + 4096 records,
    pcppx_kernels.hip flow_queue_capacity) overflows many times over. The count kernel bounds every queue write by the
    queue's capacity and adds an overflowing record to the table with device atomics (flow_region_add_atomic), the
    merge reads min(fill, capacity) records -- so the table is exact and nothing is written past the queues (the
    round-3 illegal address in tools/ab_flow_part.py was that harness's own queue buffer, sized for the product
    layout, under a variant with another layout: DESIGN.md §6)."""
    n, cap = 300_000, 1 << 21
    k = np.arange(1, 1 << 26, dtype=np.uint64)
    part = ((k * 0x9E3779B1) & 0xFFFFFFFF) >> 23
    keys = k[part == 0][: 40_000].astype(np.uint32)  # 40k distinct keys, all in partition 0 (region 4096 slots)
    assert len(keys) == 40_000
    rng = np.random.default_rng(7)
    s = np.zeros(n, dtype=abi.SUMMARY_DTYPE)
    s["hash5"] = keys[rng.integers(0, len(keys), n)]
    caplens = rng.integers(60, 1515, n).astype(np.uint32)
    got, st = _device_flow_table(engine, s, caplens, n, cap)
    want = _host_group_by(s, caplens)
    for key, v in got.items():
        assert want[key] == v, key
    # the region holds 4096 slots: the rest of the keys' packets are counted as lost, none vanish
    assert len(got) <= 4096 and sum(v[0] for v in got.values()) + int(st[2]) == n


def test_gpu_flow_table_full_conserves_packets(engine):
    """A table far smaller than the flow count: a key once stored is never displaced, so every stored
    flow's counters are exact, and stored + lost (stats[2]) + key-0 packets account for every packet."""
    b = synth.imix(500_000, 11, corrupt_frac=0.0, flows=100_000)
    s, _ = parse_on_device(engine, b, abi.make_opts(0, 8, False, 0))
    cap = 1 << 12
    got, st = _device_flow_table(engine, s, b.caplens, b.n, cap)
    want = _host_group_by(s, b.caplens)
    zero = want.pop(0, (0, 0))
    assert len(got) == cap
    for key, v in got.items():
        assert want[key] == v, key
    assert sum(v[0] for v in got.values()) + int(st[2]) + int(st[0]) == b.n
    assert int(st[0]) == zero[0] and int(st[2]) > 0


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.stem)
def test_gpu_flag_contract_parse_until(engine, path):
    """The device's NEEDS_HOST flags against the reference chain (oracle.check_flag_contract) under the full parse,
    Packet(&raw, TCP) (benchmark.cpp:91) and Packet(&raw, OsiModelNetworkLayer): a packet is flagged when the
    reference chain holds a layer the engine does not build, or the host's dissector fell back to Payload where
    the engine stopped; parse-until roll-backs of the host's layer (Packet.cpp:134-175) leave exact, unflagged
    chains."""
    batch, variants = load_golden(path)
    for v in ("full", "until_tcp", "until_osi3"):
        if v not in variants:
            continue
        opts, rsum, rlay = variants[v]
        gsum, glay = parse_on_device(engine, batch, opts)
        oracle.compare_engine_to_reference(gsum, glay, rsum, rlay)
        oracle.check_flag_contract(gsum, rsum, rlay, batch)


def test_gpu_deep_window_with_checksums(engine):
    """opts.window = PCPPX_WINDOW_DEEP (the checksum launch with the two-round 144-B header window, the tight second
    round and the dword-aligned re-gather of stacks past the window): records identical to the default window and
    to the restatement, on config-5 deep stacks with checksums (packed, so the span stream runs, and gapped, so every
    start alignment and the HBM edge-chunk path are hit) and on every golden set under its option variants."""
    b = synth.config(5, 200_000)
    deep = abi.make_opts(0, 8, True, 12, abi.WINDOW_DEEP)
    d = parse_on_device(engine, b, deep)
    dflt = parse_on_device(engine, b, abi.make_opts(0, 8, True, 12))
    oracle.compare_exact(d[0], d[1], dflt[0], dflt[1])
    has_l4 = d[0]["l4_layer"] != 0xFF  # IPv6 stacks ending in a Fragment extension carry a Payload, no L4 layer
    assert has_l4.mean() > 0.9 and ((d[0]["flags"][has_l4] & abi.F_L4_CSUM) != 0).all()
    idx = np.arange(0, b.n, 7)
    sub = from_packets([b.packet(int(i)) for i in idx])
    o = oracle.oracle_parse(sub, deep, threads=8)
    oracle.compare_exact(d[0][idx], d[1][idx], o[0], o[1])
    h = engine.parse_host(b, deep)  # the host path's chunked launches pick the same instance
    oracle.compare_exact(h[0], h[1], d[0], d[1])
    g = as_batch([b.packet(i) for i in range(30_000)], gaps=True, seed=5)
    gd = parse_on_device(engine, g, deep)
    og = oracle.oracle_parse(g, deep, threads=8)
    oracle.compare_exact(gd[0], gd[1], og[0], og[1])
    for path in golden_files():
        batch, variants = load_golden(path)
        for v, (opts, rsum, rlay) in variants.items():
            if not opts.want_checksums:
                continue
            od = abi.make_opts(opts.parse_until_family, opts.parse_until_osi, True, opts.max_layers, abi.WINDOW_DEEP)
            gs, gl = parse_on_device(engine, batch, od)
            os_, ol = oracle.oracle_parse(batch, od)
            oracle.compare_exact(gs, gl, os_, ol)


@pytest.mark.parametrize("shard_range", [(0, 12_500_000), (87_500_000, 100_000_000)], ids=["rank0of8", "rank7of8"])
def test_gpu_config4_full_size_flow_table(engine, shard_range):
    """BASELINE config 4 at its full per-GPU size on bench.py's own stream and launch: packets [lo, hi) of the one
    config-4 stream (synth.flow_stream, seed 4, 1M flows: bench.py's rank 0 of any N, and rank 7 of 8), parsed as
    bench.py parses them (the SHORT parse-only window, no layer records, the dense hash5 column and the collectStats
    counters), then three pcppx_flow_count_keys_device calls into one 2M-slot table (three bench steps). Every flow's
    {packets, bytes} equals three times a host group-by of the device keys, key 0 goes to the stats counters, nothing
    is lost; the keys equal the restatement's hash5Tuple on every packet, and the collectStats counters its own."""
    import torch

    from pcapplusplus_amd.engine import to_device

    lo, hi = shard_range
    n = hi - lo
    b = synth.flow_stream(lo, hi, 4, flows=1_000_000)
    dev = "cuda:0"
    data, offs, caps = to_device(b, dev)
    st = torch.cuda.current_stream().cuda_stream
    fk = torch.empty(n, dtype=torch.int32, device=dev)
    ps = torch.zeros(abi.PROTO_STATS, dtype=torch.int64, device=dev)
    opts = abi.make_opts(0, 8, False, 0, abi.WINDOW_SHORT)
    engine.parse_device(data, offs, caps, n, b.linktype, opts, None, None, st, fk, None, ps)
    cap = 1 << 21
    keys = torch.zeros(cap, dtype=torch.int32, device=dev)
    pk = torch.zeros(cap, dtype=torch.int64, device=dev)
    by = torch.zeros(cap, dtype=torch.int64, device=dev)
    stt = torch.zeros(4, dtype=torch.int64, device=dev)
    for _ in range(3):
        engine.flow_count_keys_device(fk, caps, n, keys, pk, by, cap, stt, st)
    torch.cuda.synchronize()
    k = keys.cpu().numpy().view(np.uint32)
    used = k != 0
    got = dict(zip(k[used].tolist(), zip(pk.cpu().numpy()[used].tolist(), by.cpu().numpy()[used].tolist())))
    hk = fk.cpu().numpy().view(np.uint32)
    pstats = ps.cpu().numpy()
    del data, offs, caps, fk, keys, pk, by, ps
    uk, inv = np.unique(hk, return_inverse=True)
    cnt = np.bincount(inv)
    byt = np.bincount(inv, weights=b.caplens.astype(np.float64)).astype(np.int64)
    want = {int(x): (3 * int(c), 3 * int(y)) for x, c, y in zip(uk.tolist(), cnt.tolist(), byt.tolist()) if x != 0}
    z = int(cnt[0]) if uk[0] == 0 else 0
    zb = int(byt[0]) if uk[0] == 0 else 0
    assert len(want) > 400_000
    assert got == want
    s = stt.cpu().numpy()
    assert (int(s[0]), int(s[1]), int(s[2])) == (3 * z, 3 * zb, 0)
    o = oracle.oracle_parse(b, abi.make_opts(0, 8, False, 0), threads=16)
    assert np.array_equal(hk, o[0]["hash5"])
    assert {f: int(pstats[k]) for k, f in enumerate(abi.PROTO_STATS_FIELDS)} == oracle.proto_stats(o[0])
