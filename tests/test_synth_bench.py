"""Synthetic workloads (pcapplusplus_amd/synth.py) and the bench's byte model, on CPU.

The config generators must produce exactly the stacks SURVEY.md §8d names, parse with no host fallback and
carry valid checksums (the restatement checks them); bench.py's header-extent byte model (parse-only runs)
must equal the same quantity computed from the restatement's records.
"""
from __future__ import annotations

import sys

import numpy as np
import pytest

import oracle
from conftest import ROOT
from pcapplusplus_amd import abi, synth

P_ETH, P_IPV4, P_IPV6, P_TCP, P_UDP, P_VLAN, P_MPLS, P_GREV0, P_PAYLOAD = 1, 2, 3, 4, 5, 9, 14, 15, 25


def has(mask, p):
    return ((mask >> np.uint64(p)) & np.uint64(1)).astype(bool)


def test_config5_stack_mix_and_checksums():
    b = synth.config(5, 20_000)
    s, lay = oracle.oracle_parse(b, abi.make_opts(0, 8, True, 16), threads=8)
    fl = s["flags"]
    assert not (fl & (abi.F_NEEDS_HOST | abi.F_DEPTH_OVERFLOW | abi.F_TRAILER)).any()
    m = s["proto_mask"]
    n = b.n
    # every stack kind is present in roughly the generator's proportions
    assert 0.25 < has(m, P_MPLS).mean() < 0.35
    assert 0.25 < has(m, P_GREV0).mean() < 0.35
    assert has(m, P_VLAN).mean() > 0.6
    # QinQ: two VLAN layers in about half the packets
    nv = (lay["proto"] == P_VLAN).sum(axis=1)
    assert 0.4 < (nv == 2).mean() < 0.6
    # IPv6 extension chains: IPv6 header length > 40 somewhere
    v6ext = ((lay["proto"] == P_IPV6) & (lay["hdr_len"] > 40)).any(axis=1)
    assert 0.25 < v6ext.mean() < 0.35
    # valid checksums wherever an L4 layer is parsed (no corruption in config 5)
    l4 = (fl & abi.F_L4_CSUM) != 0
    assert l4.mean() > 0.9 and ((fl[l4] & abi.F_L4_CSUM_OK) != 0).all()
    ip = (fl & abi.F_IP_CSUM) != 0
    assert ((fl[ip] & abi.F_IP_CSUM_OK) != 0).all()
    # chains end in Payload and cover the packet
    nl = s["n_layers"].astype(np.int64)
    last = lay[np.arange(n), nl - 1]
    assert (last["proto"] == P_PAYLOAD).all()
    assert (last["offset"].astype(np.int64) + last["data_len"] == b.caplens).all()


@pytest.mark.parametrize("cfg,n", [(1, 2000), (2, 5000), (3, 20_000), (4, 20_000)])
def test_configs_parse_without_host_fallback(cfg, n):
    b = synth.config(cfg, n)
    s, _ = oracle.oracle_parse(b, abi.make_opts(0, 8, True, 8), threads=8)
    assert not (s["flags"] & abi.F_NEEDS_HOST).any()
    l4 = (s["flags"] & abi.F_L4_CSUM) != 0
    ok = (s["flags"] & abi.F_L4_CSUM_OK) != 0
    bad = int((l4 & ~ok).sum())
    if cfg == 3:
        assert bad > 0  # 1% corrupted checksums (half of them L4)
    else:
        assert bad == 0


@pytest.mark.parametrize("cfg", [2, 5])
def test_bench_header_extent_byte_model(cfg):
    """bench.algorithmic_read_bytes (torch over the records) == the extent computed here in numpy."""
    import torch

    sys.path.insert(0, str(ROOT))
    import bench

    b = synth.config(cfg, 3000)
    ml = 12
    s, lay = oracle.oracle_parse(b, abi.make_opts(0, 8, False, ml))
    got = bench.algorithmic_read_bytes(b, False, torch.from_numpy(s.view(np.uint8).copy()),
                                       torch.from_numpy(lay.view(np.uint8).reshape(-1).copy()),
                                       torch.from_numpy(b.caplens.view(np.int32).copy()), ml)
    nl = s["n_layers"].astype(np.int64)
    end = lay["offset"].astype(np.int64) + lay["hdr_len"]
    valid = (np.arange(ml)[None, :] < nl[:, None]) & (lay["proto"] != P_PAYLOAD) & (lay["proto"] != 30)
    ext = np.minimum(np.where(valid, end, 0).max(axis=1), b.caplens)
    assert got == int(ext.sum()) + 12 * b.n
    assert bench.algorithmic_read_bytes(b, True) == int(b.caplens.sum(dtype=np.int64)) + 12 * b.n


def test_flow_stream_ranges_are_one_stream():
    """BASELINE config 4 is ONE stream over ONE flow universe cut into contiguous shards: any range
    of synth.flow_stream carries the same caplens, flows and hash5Tuple keys as that range of a longer call, across
    block boundaries, and shards share flows."""
    import numpy as np

    import oracle
    from pcapplusplus_amd import abi, synth

    blk = synth.FLOW_STREAM_BLOCK
    lo, hi = blk - 20_000, blk + 30_000
    whole = synth.flow_stream(0, hi, 4, flows=5000)
    part = synth.flow_stream(lo, hi, 4, flows=5000)
    assert part.n == hi - lo
    assert np.array_equal(part.caplens, whole.caplens[lo:hi])
    assert np.array_equal(part.meta["flow_id"], whole.meta["flow_id"][lo:hi])
    opts = abi.make_opts(0, 8, False, 0)
    sp, _ = oracle.oracle_parse(part, opts, threads=8)
    sw, _ = oracle.oracle_parse(whole.slice(lo, hi), opts, threads=8)
    assert np.array_equal(sp["hash5"], sw["hash5"]) and (sp["hash5"] != 0).all()
    a = set(synth.flow_stream(0, 20_000, 4, flows=5000).meta["flow_id"].tolist())
    b = set(synth.flow_stream(20_000, 40_000, 4, flows=5000).meta["flow_id"].tolist())
    assert len(a & b) > 500  # the Zipf head: flows span shards
    assert synth.config(4, 1000).meta["stream_lo"] == 0
