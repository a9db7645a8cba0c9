"""The restatement against the LIVE reference on adversarial inputs (mutations + crafted deep stacks).

Needs oracle/_ref/libpcpp_ref.so (the reference compiled from /root/reference by oracle/Makefile);
skipped where it was not built.
"""
from __future__ import annotations

import pytest

import oracle
from conftest import golden_files, load_golden
from mutate import as_batch, crafted, crafted_l7, mutate
from pcapplusplus_amd import abi

pytestmark = pytest.mark.skipif(not oracle.ref_available(), reason="reference library not built")

OPTS = [abi.make_opts(), abi.make_opts(4, 8, True, 16), abi.make_opts(0, 3, True, 16),
        abi.make_opts(0x203, 8, True, 4), abi.make_opts(0, 8, True, 0), abi.make_opts(0, 4, True, 16),
        abi.make_opts(0, 5, True, 16), abi.make_opts(0, 6, True, 16), abi.make_opts(5, 8, True, 16),
        abi.make_opts(0x607, 8, True, 16), abi.make_opts(18, 8, True, 16), abi.make_opts(13, 8, True, 16),
        abi.make_opts(0, 7, True, 8), abi.make_opts(0x1219, 8, True, 16)]


def _seed_packets():
    batch, _ = load_golden([p for p in golden_files() if p.stem == "pcap_lt1"][0])
    dat, _ = load_golden([p for p in golden_files() if p.stem == "dat_ethernet"][0])
    return [batch.packet(i) for i in range(0, batch.n, 3)] + [dat.packet(i) for i in range(dat.n)]


@pytest.mark.parametrize("opt_i", range(len(OPTS)))
def test_crafted_stacks_vs_reference(opt_i):
    b = as_batch(crafted())
    rs, rl = oracle.ref_parse(b, OPTS[opt_i])
    os_, ol = oracle.oracle_parse(b, OPTS[opt_i])
    oracle.compare_engine_to_reference(os_, ol, rs, rl)
    if OPTS[opt_i].max_layers >= 8:
        oracle.check_flag_contract(os_, rs, rl, b)


@pytest.mark.parametrize("opt_i", range(len(OPTS)))
def test_crafted_l7_payloads_vs_reference(opt_i):
    """The L7 content checks (HTTP / SSL / DNS first layers; plain Payload otherwise) at their edges."""
    b = as_batch(crafted_l7())
    rs, rl = oracle.ref_parse(b, OPTS[opt_i])
    os_, ol = oracle.oracle_parse(b, OPTS[opt_i])
    oracle.compare_engine_to_reference(os_, ol, rs, rl)
    if OPTS[opt_i].max_layers >= 8:
        st = oracle.check_flag_contract(os_, rs, rl, b)
        if opt_i == 0:
            assert st["l7_known"] > 0 and st["flagged"] < b.n


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mutations_vs_reference(seed):
    b = as_batch(mutate(_seed_packets(), 6000, seed), gaps=True, seed=seed)
    for opts in OPTS[:3] + OPTS[5:]:
        rs, rl = oracle.ref_parse(b, opts)
        os_, ol = oracle.oracle_parse(b, opts)
        oracle.compare_engine_to_reference(os_, ol, rs, rl)
        oracle.check_flag_contract(os_, rs, rl, b)


@pytest.mark.parametrize("linktype", [0, 113, 276, 104, 239])
def test_link_layers_vs_reference(linktype):
    """Linux SLL / SLL2 / Null-Loopback / Cisco HDLC / NFLOG first layers (Packet::createFirstLayer, Packet.cpp:827-923): crafted edge
    cases and mutations of the reference's own captures of that link type."""
    from mutate import crafted_linklayers
    from pcapplusplus_amd.pcap import from_packets

    seeds = crafted_linklayers()[linktype]
    g = [p for p in golden_files() if p.stem == f"pcap_lt{linktype}"]
    if g:
        gb, _ = load_golden(g[0])
        seeds = seeds + [gb.packet(i) for i in range(gb.n)]
    b = from_packets(seeds + mutate(seeds, 3000, linktype + 1), linktype)
    for opts in OPTS[:4] + OPTS[5:]:
        rs, rl = oracle.ref_parse(b, opts)
        os_, ol = oracle.oracle_parse(b, opts)
        oracle.compare_engine_to_reference(os_, ol, rs, rl)
        if opts.max_layers >= 8:
            oracle.check_flag_contract(os_, rs, rl, b)
    s, _ = oracle.oracle_parse(b, OPTS[0])
    assert ((s["flags"] & abi.F_NEEDS_HOST) == 0).mean() > 0.5
