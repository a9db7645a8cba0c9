"""ABI 7: the 16-B brief (pcppx_records.brief, the summary's first half) and the host path's DENSE layer layout
(PCPPX_LAYOUT_DENSE: the chains back to back over the batch, pcppx_records.layers_written of them).

CPU: the ctypes / numpy mirrors match the header (sizes, offsets), the DENSE positions decode a known layout, and
pcppx_chain_proto_mask over the restatement's rows equals its summary proto_mask wherever the chain is recorded whole
(every golden set: the brief's isPacketOfType is exact there).
GPU: a brief written beside a summary is the summary's first 16 bytes on every packet (configs 3 and 5, checksums on and
off, FIXED and PACKED rows, every golden set, gapped batches); a brief-only launch writes the same rows (PACKED decoded
through the brief); the host path's DENSE rows (pageable and page-locked outputs, more than one 256k-packet chunk, gapped
batches, brief or summary as the length source) decode to the FIXED rows, with layers_written their total.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import oracle
from conftest import golden_files, load_golden
from pcapplusplus_amd import abi, synth


def test_abi7_structs():
    assert abi.ABI_VERSION == 7 and abi.BRIEF_DTYPE.itemsize == 16
    assert abi.BRIEF_DTYPE.names == abi.SUMMARY_DTYPE.names[:6]
    assert C.sizeof(abi.Records) == 64 and abi.Records.brief.offset == 48 and abi.Records.layers_written.offset == 56
    s = np.zeros(3, abi.SUMMARY_DTYPE)
    s["hash5"], s["flags"], s["n_layers"], s["l4_layer"], s["proto_mask"] = [1, 2, 3], 0x41, [4, 5, 6], 2, 99
    b = s.view(np.uint8).reshape(3, 32)[:, :16].copy().view(abi.BRIEF_DTYPE).ravel()
    for f in abi.BRIEF_DTYPE.names:
        assert (b[f] == s[f]).all()


def test_dense_positions_decode():
    nl = np.array([3, 0, 5, 16, 2], np.uint8)
    ml = 4
    pos = abi.dense_positions(nl, ml)
    assert pos.tolist() == [0, 3, 3, 7, 11]
    fixed = np.zeros((5, ml), abi.LAYER_DTYPE)
    for i, c in enumerate(np.minimum(nl, ml)):
        fixed["proto"][i, :c] = np.arange(1, c + 1) + 10 * i
    dense = np.concatenate([fixed[i, :min(int(nl[i]), ml)] for i in range(5)])
    assert len(dense) == 13
    back = abi.unpack_dense(nl, dense, ml)
    assert back.tobytes() == fixed.tobytes()


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.stem)
def test_chain_proto_mask_equals_summary_mask(path):
    """isPacketOfType from the recorded rows (what a brief's reader computes) equals the summary's proto_mask on every
    packet whose chain is recorded whole (16 layers, no depth overflow)."""
    batch, _ = load_golden(path)
    for fam, osi in ((0, 8), (4, 8), (0, 3)):
        s, lay = oracle.oracle_parse(batch, abi.make_opts(fam, osi, False, 16))
        whole = (s["flags"] & abi.F_DEPTH_OVERFLOW) == 0
        m = abi.chain_proto_mask(lay, s["n_layers"])
        assert (m[whole] == s["proto_mask"][whole]).all(), (path.stem, fam, osi)


def _brief_of(summary: np.ndarray) -> np.ndarray:
    return summary.view(np.uint8).reshape(len(summary), 32)[:, :16].copy().view(abi.BRIEF_DTYPE).ravel()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,ml,csum,layout", [(3, 8, True, abi.LAYOUT_PACKED), (3, 8, True, abi.LAYOUT_FIXED),
                                                (5, 12, False, abi.LAYOUT_PACKED), (5, 12, True, abi.LAYOUT_PACKED),
                                                (4, 0, False, abi.LAYOUT_FIXED), (2, 16, False, abi.LAYOUT_FIXED)])
def test_gpu_brief_is_the_summary_half(engine, cfg, ml, csum, layout):
    from mutate import as_batch

    from pcapplusplus_amd.engine import parse_on_device_ex

    b = synth.config(cfg, 100_000)
    o = abi.make_opts(0, 8, csum, ml, layout=layout)
    both = parse_on_device_ex(engine, b, o, brief=True)
    assert both["brief"].tobytes() == _brief_of(both["summary"]).tobytes()
    only = parse_on_device_ex(engine, b, o, summary=False, brief=True)
    assert only["brief"].tobytes() == both["brief"].tobytes()
    if ml:
        assert only["layers"].tobytes() == both["layers"].tobytes()
        whole = (both["summary"]["flags"] & abi.F_DEPTH_OVERFLOW) == 0
        m = abi.chain_proto_mask(only["layers"], only["brief"]["n_layers"])
        assert (m[whole] == both["summary"]["proto_mask"][whole]).all()
    os_, ol = oracle.oracle_parse(b, abi.make_opts(0, 8, csum, ml))
    oracle.compare_exact(both["summary"], both["layers"] if ml else ol, os_, ol)
    g = as_batch([b.packet(i) for i in range(0, b.n, 7)], gaps=True, seed=cfg)
    gb = parse_on_device_ex(engine, g, o, brief=True)
    assert gb["brief"].tobytes() == _brief_of(gb["summary"]).tobytes()


@pytest.mark.gpu
def test_gpu_brief_golden(engine):
    from pcapplusplus_amd.engine import parse_on_device_ex

    for path in golden_files():
        batch, variants = load_golden(path)
        for v, (opts, _, _) in variants.items():
            g = parse_on_device_ex(engine, batch, opts, brief=True)
            assert g["brief"].tobytes() == _brief_of(g["summary"]).tobytes(), (path.stem, v)


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("src", ["brief", "summary"])
def test_gpu_host_dense_layout(engine, pinned, src):
    """pcppx_parse_batch_host with PCPPX_LAYOUT_DENSE: the chains back to back (across 256k-packet chunks) decode to the
    FIXED rows of the same parse; layers_written is their total; a gapped batch and every golden set too."""
    from mutate import as_batch

    b = synth.config(3, 600_000)  # three chunks of the host path
    for ml, csum in ((16, False), (8, True)):
        fo = abi.make_opts(0, 8, csum, ml)
        fs, fl = engine.parse_host(b, fo)
        do = abi.make_opts(0, 8, csum, ml, layout=abi.LAYOUT_DENSE)
        s, br, dense, w = engine.parse_host_ex(b, do, want_summary=src == "summary", want_brief=src == "brief",
                                               pinned=pinned)
        nl = (s if s is not None else br)["n_layers"]
        assert w == int(np.minimum(fs["n_layers"], ml).sum()) == len(dense)
        assert abi.unpack_dense(nl, dense, ml).tobytes() == np.where(
            np.arange(ml)[None, :] < np.minimum(fs["n_layers"], ml)[:, None], fl, np.zeros(1, abi.LAYER_DTYPE)).tobytes()
        if s is not None:
            assert s.tobytes() == fs.tobytes()
        else:
            assert br.tobytes() == _brief_of(fs).tobytes()
    g = as_batch([b.packet(i) for i in range(0, 100_000, 3)], gaps=True, seed=5)
    o = abi.make_opts(0, 8, False, 16, layout=abi.LAYOUT_DENSE)
    _, br, dense, w = engine.parse_host_ex(g, o, want_summary=False, want_brief=True, pinned=pinned)
    os_, ol = oracle.oracle_parse(g, abi.make_opts(0, 8, False, 16))
    oracle.compare_exact(os_, abi.unpack_dense(br["n_layers"], dense, 16), os_, ol)
    assert br.tobytes() == _brief_of(os_).tobytes()
    for path in golden_files()[:6]:
        batch, variants = load_golden(path)
        for v, (opts, _, _) in variants.items():
            o = abi.make_opts(opts.parse_until_family, opts.parse_until_osi, bool(opts.want_checksums), opts.max_layers,
                              layout=abi.LAYOUT_DENSE)
            _, br, dense, w = engine.parse_host_ex(batch, o, want_summary=False, want_brief=True, pinned=pinned)
            os_, ol = oracle.oracle_parse(batch, opts)
            assert br.tobytes() == _brief_of(os_).tobytes(), (path.stem, v)
            oracle.compare_exact(os_, abi.unpack_dense(br["n_layers"], dense, opts.max_layers), os_, ol)


@pytest.mark.gpu
def test_gpu_engine_window_choice():
    """PCPPX_WINDOW_DEFAULT is the engine's choice (ABI 7): after parsing deep stacks (config 5) a context runs checksum
    launches with the two-round window (as WINDOW_DEEP) and keeps the second round for parse-only ones; after plain
    stacks (config 3) it runs parse-only launches as SHORT and checksum launches with the one 96-B window. The records are
    the restatement's whatever was chosen (device and host paths)."""
    from pcapplusplus_amd.engine import Engine, parse_on_device

    for cfg, want_csum_win, want_po_win in ((5, abi.WINDOW_DEEP, abi.WINDOW_DEFAULT),
                                            (3, abi.WINDOW_DEFAULT, abi.WINDOW_SHORT)):
        b = synth.config(cfg, 200_000)
        with Engine(0) as eng:
            assert eng.window_choice(True) == abi.WINDOW_DEFAULT  # nothing sampled yet
            for csum in (True, False, True):
                o = abi.make_opts(0, 8, csum, 12 if cfg == 5 else 8)
                s, lay = parse_on_device(eng, b, o)
                if csum:
                    os_, ol = oracle.oracle_parse(b, o, threads=8)
                    oracle.compare_exact(s, lay, os_, ol)
            assert eng.window_choice(True) == want_csum_win, cfg
            assert eng.window_choice(False) == want_po_win, cfg
            hs, hl = eng.parse_host(b, abi.make_opts(0, 8, True, 8))  # the host path follows the same choice
            os_, ol = oracle.oracle_parse(b, abi.make_opts(0, 8, True, 8), threads=8)
            oracle.compare_exact(hs, hl, os_, ol)
    # parses whose window the caller forces are not sampled: a context that only ran those has decided nothing
    with Engine(0) as eng:
        b = synth.config(5, 200_000)
        for w in (abi.WINDOW_SHORT, abi.WINDOW_DEEP, abi.WINDOW_SHORT):
            parse_on_device(eng, b, abi.make_opts(0, 8, w == abi.WINDOW_DEEP, 12, w))
        assert eng.window_choice(True) == abi.WINDOW_DEFAULT and eng.window_choice(False) == abi.WINDOW_DEFAULT


@pytest.mark.gpu
def test_gpu_host_path_empty_reset_and_dense_limit(engine):
    """pcppx_parse_batch_host: an empty batch resets a reused records struct's layout and layers_written
    before returning OK; a DENSE batch whose n * max_layers exceeds the 32-bit entry positions is refused with
    PCPPX_E_INVAL before any memory is touched (the 64-B buffers below stand in for a 268M-packet batch and are never
    read)."""
    lib = engine.lib
    buf = np.zeros(64, dtype=np.uint8)
    p = buf.ctypes.data
    opts = abi.make_opts(0, 8, False, 16, layout=abi.LAYOUT_DENSE)
    rec = abi.Records(p, p, None, None)
    rec.layout, rec.layers_written = 0, 12345
    empty = abi.Batch(p, p, p, 64, 0, 1, 0)
    assert lib.pcppx_parse_batch_host(engine.ctx, C.byref(empty), C.byref(opts), C.byref(rec)) == 0
    assert rec.layers_written == 0 and rec.layout == abi.LAYOUT_DENSE
    huge = abi.Batch(p, p, p, 64, (1 << 32) // 16 + 1, 1, 0)  # 268,435,457 packets x 16 entries > UINT32_MAX
    rec.layers_written = 777
    assert lib.pcppx_parse_batch_host(engine.ctx, C.byref(huge), C.byref(opts), C.byref(rec)) == abi.E_INVAL
    assert rec.layers_written == 0
