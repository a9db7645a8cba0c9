"""Reassembly front ends: pcppx_reasm_device and its restatement.

The stateless per-packet half of IPReassembly::processPacket (Packet++/src/IPReassembly.cpp:281-322) and
TcpReassembly::reassemblePacket (Packet++/src/TcpReassembly.cpp:81-141): status, fragment key
(hashPacket, IPReassembly.cpp:103-115/190-205), fragment id / offset / first / last, TCP payload size and
SYN/FIN/RST. Bar: bit-exact.

CPU: the restatement (oracle_reasm over the restatement's parse records) equals the real reference run on
a first sighting (oracle/ref_harness.cpp: pcppx_ref_reasm) and the frozen golden vectors
(tests/golden/reasm/, tools/make_golden_reasm.py) on every packet whose status the engine decides
(statuses *_HOST leave the packet to the host).
GPU: the device path equals the restatement on every field of every packet (HOST statuses included).
"""
from __future__ import annotations


import numpy as np
import pytest

import oracle
from conftest import GOLDEN, golden_files, load_golden
from mutate import as_batch, fragments, mutate
from pcapplusplus_amd import abi
from pcapplusplus_amd.pcap import PacketBatch

OPTS = abi.make_opts(0, 8, False, 16)
REASM_GOLDEN = GOLDEN / "reasm"


def decided(info):
    """(ip decided, tcp decided) masks: packets whose status the engine settles on the device."""
    return (info["ip_status"] & 0xF) != abi.IPR_HOST, (info["tcp_status"] & 0xF) != abi.TCPR_HOST


def compare_to_reference(eng, ref, what: str) -> dict:
    ipd, tcd = decided(eng)
    for f in ("ip_status", "ip_key", "frag_id", "frag_offset"):
        bad = np.nonzero(ipd & (eng[f] != ref[f]))[0]
        assert len(bad) == 0, (what, f, len(bad), eng[bad[0]], ref[bad[0]])
    for f in ("tcp_status", "tcp_payload"):
        bad = np.nonzero(tcd & (eng[f] != ref[f]))[0]
        assert len(bad) == 0, (what, f, len(bad), eng[bad[0]], ref[bad[0]])
    return {"n": len(eng), "ip_decided": int(ipd.sum()), "tcp_decided": int(tcd.sum()),
            "fragments": int(((eng["ip_status"] & 0xF) == abi.IPR_FRAGMENT).sum())}


def golden_reasm():
    """(name, batch, reference info) for every frozen reassembly golden set."""
    out = []
    parse_sets = {p.stem: p for p in golden_files()}
    for p in sorted(REASM_GOLDEN.glob("*.npz")):
        z = np.load(p, allow_pickle=False)
        if "data" in z.files:
            b = PacketBatch(z["data"], z["offsets"], z["caplens"], int(z["linktype"]))
        else:
            b, _ = load_golden(parse_sets[p.stem])
        out.append((p.stem, b, z["info"]))
    return out


def restated(batch, opts=OPTS):
    s, lay = oracle.oracle_parse(batch, opts)
    return oracle.oracle_reasm(batch, s, lay)


# ---------------------------------------------------------------- CPU: restatement vs reference
@pytest.mark.parametrize("name,batch,ref", golden_reasm(), ids=lambda x: x if isinstance(x, str) else "")
def test_restatement_matches_golden(name, batch, ref):
    st = compare_to_reference(restated(batch), ref, name)
    assert st["ip_decided"] > 0.8 * st["n"]
    if name == "fragments":
        assert st["fragments"] > 1000


def test_golden_sets_cover_every_status():
    """The pinned vectors exercise every status and flag the restatement emits."""
    infos = np.concatenate([ref for _, _, ref in golden_reasm()])
    ips, ts = infos["ip_status"], infos["tcp_status"]
    for code in (abi.IPR_NON_IP, abi.IPR_NON_FRAGMENT, abi.IPR_MALFORMED, abi.IPR_FRAGMENT):
        assert ((ips & 0xF) == code).any(), code
    for fl in (abi.IPR_F_FIRST, abi.IPR_F_LAST, abi.IPR_F_IPV6):
        assert ((ips & fl) != 0).any(), fl
    for code in (abi.TCPR_NON_IP, abi.TCPR_NON_TCP, abi.TCPR_NO_DATA, abi.TCPR_DATA):
        assert ((ts & 0xF) == code).any(), code
    for fl in (abi.TCPR_F_FIN, abi.TCPR_F_SYN, abi.TCPR_F_RST):
        assert ((ts & fl) != 0).any(), fl


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build absent")
@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.stem)
def test_restatement_matches_reference_fixtures(path):
    batch, _ = load_golden(path)
    compare_to_reference(restated(batch), oracle.ref_reasm(batch), path.stem)


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build absent")
@pytest.mark.parametrize("seed", [13, 14])
def test_restatement_matches_reference_fragments(seed):
    pk = fragments(6000, seed)
    for b in (as_batch(pk), as_batch(mutate(pk, 6000, seed))):
        for opts in (OPTS, abi.make_opts(0, 8, False, 4)):  # shallow records: DEPTH_OVERFLOW -> host
            compare_to_reference(restated(b, opts), oracle.ref_reasm(b), f"fragments seed {seed}")


# ---------------------------------------------------------------- device
def gpu_reasm(engine, batch, max_layers=16):
    import torch

    from pcapplusplus_amd.engine import to_device

    dev = "cuda:0"
    n = batch.n
    data, offsets, caplens = to_device(batch, dev)
    summary = torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device=dev)
    layers = torch.zeros(max(n * max_layers, 1) * 8, dtype=torch.uint8, device=dev)
    info = torch.full((max(n, 1) * 16,), 0xAB, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    engine.parse_device(data, offsets, caplens, n, batch.linktype, abi.make_opts(0, 8, False, max_layers), summary,
                        layers, stream)
    engine.reasm_device(data, offsets, caplens, n, batch.linktype, summary, layers, max_layers, info, stream)
    torch.cuda.synchronize(dev)
    return info.cpu().numpy().view(abi.REASM_DTYPE)[:n]


def assert_equal_info(a, b, what):
    for f in a.dtype.names:
        bad = np.nonzero(a[f] != b[f])[0]
        assert len(bad) == 0, (what, f, len(bad), a[bad[0]], b[bad[0]])


@pytest.mark.gpu
@pytest.mark.parametrize("name,batch,ref", golden_reasm(), ids=lambda x: x if isinstance(x, str) else "")
def test_gpu_reasm_golden(engine, name, batch, ref):
    g = gpu_reasm(engine, batch)
    assert_equal_info(g, restated(batch), name)
    compare_to_reference(g, ref, name)


@pytest.mark.gpu
@pytest.mark.parametrize("max_layers", [16, 4])
def test_gpu_reasm_fragments_and_mutations(engine, max_layers):
    pk = fragments(20000, 41)
    for b in (as_batch(pk, gaps=True, seed=2), as_batch(mutate(pk, 20000, 8))):
        g = gpu_reasm(engine, b, max_layers)
        assert_equal_info(g, restated(b, abi.make_opts(0, 8, False, max_layers)), "fragments")
        if oracle.ref_available():
            compare_to_reference(g, oracle.ref_reasm(b), "fragments")


@pytest.mark.gpu
def test_gpu_reasm_all_parse_fixtures(engine):
    for p in golden_files():
        b, _ = load_golden(p)
        assert_equal_info(gpu_reasm(engine, b), restated(b), p.stem)


@pytest.mark.gpu
def test_gpu_reasm_rejects_bad_args(engine):
    import torch

    t = torch.zeros(64, dtype=torch.int64, device="cuda:0")
    with pytest.raises(RuntimeError):  # max_layers 0: no records to read the IP/TCP layers from
        engine.reasm_device(t, t, t, 4, 1, t, t, 0, t)
    with pytest.raises(RuntimeError):
        engine.reasm_device(t, t, t, 4, 1, t, t, 17, t)


def gpu_parse_reasm_fused(engine, batch, opts):
    """pcppx_parse_batch_device_reasm: records and reassembly info from one kernel pass."""
    import torch

    from pcapplusplus_amd.engine import records_from_device, to_device

    dev = "cuda:0"
    n = batch.n
    data, offsets, caplens = to_device(batch, dev)
    summary = torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device=dev)
    layers = torch.zeros(max(n * opts.max_layers, 1) * 8, dtype=torch.uint8, device=dev)
    info = torch.full((max(n, 1) * 16,), 0xAB, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    engine.parse_reasm_device(data, offsets, caplens, n, batch.linktype, opts, summary, layers, info, stream)
    torch.cuda.synchronize(dev)
    s, lay = records_from_device(summary, layers, n, opts.max_layers)
    return s, lay, info.cpu().numpy().view(abi.REASM_DTYPE)[:n]


@pytest.mark.gpu
@pytest.mark.parametrize("ml,csum", [(16, False), (8, True), (4, False)])
def test_gpu_fused_parse_reasm(engine, ml, csum):
    """The fused pass equals the parse + pcppx_reasm_device pair and the restatement, records included."""
    from pcapplusplus_amd import synth
    from pcapplusplus_amd.pcap import concat

    opts = abi.make_opts(0, 8, csum, ml)
    pk = fragments(8000, 77)
    sets = [as_batch(pk), as_batch(mutate(pk, 8000, 9), gaps=True, seed=4), synth.config(3, 20000),
            synth.config(5, 20000)] + [load_golden(p)[0] for p in golden_files() if p.stem in ("pcap_lt1", "dat_ethernet")]
    for b in sets:
        s, lay, info = gpu_parse_reasm_fused(engine, b, opts)
        os_, ol = oracle.oracle_parse(b, opts)
        oracle.compare_exact(s, lay, os_, ol)
        assert_equal_info(info, oracle.oracle_reasm(b, os_, ol), "fused")
        assert_equal_info(info, gpu_reasm(engine, b, ml), "fused vs separate")


@pytest.mark.gpu
def test_gpu_fused_parse_reasm_rejects_bad_args(engine):
    import torch

    t = torch.zeros(64, dtype=torch.int64, device="cuda:0")
    with pytest.raises(RuntimeError):  # max_layers 0: the fused pass needs layer records
        engine.parse_reasm_device(t, t, t, 4, 1, abi.make_opts(0, 8, False, 0), t, t, t)
