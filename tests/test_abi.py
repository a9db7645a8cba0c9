"""The C-ABI library loads (no GPU needed) and exports every function include/pcppx.h declares;
record layouts of the header match the Python/numpy mirror."""
from __future__ import annotations

import ctypes as C
import re
import subprocess
import tempfile
from pathlib import Path

import pytest

from pcapplusplus_amd import abi

HEADER = abi.REPO_DIR / "include" / "pcppx.h"


def declared_functions() -> list[str]:
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"^PCPPX_API\s+(?:int|void|void\*|uint32_t|const char\*)\s+(pcppx_\w+)\s*\(", txt,
                                 flags=re.M)))


def test_header_declares_expected_api():
    assert declared_functions() == sorted(abi.EXPORTED_SYMBOLS)


def test_engine_library_exports_every_symbol():
    if not abi.ENGINE_SO.exists():
        pytest.fail("libpcppx.so not built (run __graft_entry__.build())")
    lib = C.CDLL(str(abi.ENGINE_SO))
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    lib.pcppx_abi_version.restype = C.c_int
    assert lib.pcppx_abi_version() == abi.ABI_VERSION


def test_engine_library_exports_only_the_header_api():
    """Hidden visibility: the product library exports exactly include/pcppx.h (no A/B or launcher symbols)."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(abi.ENGINE_SO)], capture_output=True, text=True,
                         check=True).stdout
    names = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    ours = sorted(n for n in names if "pcppx" in n)
    assert ours == declared_functions()


def test_product_sources_read_no_environment():
    """No runtime knobs: the kernel / launch shapes are fixed in the product library (A/B shapes live in
    tools/ab/)."""
    csrc = abi.PKG_DIR / "csrc"
    for f in list(csrc.glob("*.hip")) + list(csrc.glob("*.cpp")):
        assert "getenv" not in f.read_text(), f


def test_engine_rejects_bad_arguments_without_gpu():
    lib = abi.load_engine()
    assert lib.pcppx_parse_batch_device(None, None, None, None, None) == abi.E_INVAL
    assert lib.pcppx_parse_batch_host(None, None, None, None) == abi.E_INVAL
    o = abi.Opts()
    lib.pcppx_default_opts(C.byref(o))
    assert (o.parse_until_family, o.parse_until_osi, o.want_checksums, o.max_layers) == (0, 8, 1, 16)
    assert lib.pcppx_strerror(abi.E_INVAL) == b"invalid argument"
    o.window = 3  # PCPPX_WINDOW_DEFAULT / DEEP / SHORT only
    b = abi.Batch(1, 1, 1, 1, 1, 1, 0)
    r = abi.Records(1, 1)
    assert lib.pcppx_parse_batch_device(C.c_void_p(1), C.byref(b), C.byref(o), C.byref(r), None) == abi.E_INVAL


def test_struct_layout_matches_header():
    src = r"""
    #include <stdio.h>
    #include <stddef.h>
    #include "pcppx.h"
    #define F(T, f) printf(#T "." #f " %zu %zu\n", offsetof(T, f), sizeof(((T*)0)->f));
    int main(void) {
      printf("pcppx_summary %zu\npcppx_layer %zu\npcppx_batch %zu\npcppx_opts %zu\n", sizeof(pcppx_summary),
             sizeof(pcppx_layer), sizeof(pcppx_batch), sizeof(pcppx_opts));
      F(pcppx_summary, hash5) F(pcppx_summary, hash5_dir) F(pcppx_summary, hash2) F(pcppx_summary, flags)
      F(pcppx_summary, n_layers) F(pcppx_summary, l4_layer) F(pcppx_summary, proto_mask)
      F(pcppx_summary, ip_csum_calc) F(pcppx_summary, ip_csum_stored) F(pcppx_summary, l4_csum_calc)
      F(pcppx_summary, l4_csum_stored)
      F(pcppx_layer, proto) F(pcppx_layer, osi) F(pcppx_layer, offset) F(pcppx_layer, hdr_len) F(pcppx_layer, data_len)
      return 0; }
    """
    with tempfile.TemporaryDirectory() as d:
        c = Path(d) / "l.c"
        c.write_text(src)
        exe = Path(d) / "l"
        subprocess.run(["gcc", "-I", str(HEADER.parent), str(c), "-o", str(exe)], check=True)
        out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    sizes = dict(l.split() for l in out[:4])
    assert int(sizes["pcppx_summary"]) == abi.SUMMARY_DTYPE.itemsize
    assert int(sizes["pcppx_layer"]) == abi.LAYER_DTYPE.itemsize
    assert int(sizes["pcppx_batch"]) == C.sizeof(abi.Batch)
    assert int(sizes["pcppx_opts"]) == C.sizeof(abi.Opts)
    for line in out[4:]:
        if not line:
            continue
        name, off, size = line.split()
        t, f = name.split(".")
        dt = abi.SUMMARY_DTYPE if t == "pcppx_summary" else abi.LAYER_DTYPE
        assert dt.fields[f][1] == int(off), name
        assert dt.fields[f][0].itemsize == int(size), name


def test_records_struct_matches_header():
    """pcppx_records (ABI 6: + layout) is laid out as the ctypes mirror."""
    src = r"""
    #include <stdio.h>
    #include <stddef.h>
    #include "pcppx.h"
    int main(void) { printf("%zu %zu %zu\n", sizeof(pcppx_records), offsetof(pcppx_records, layout),
                            offsetof(pcppx_records, proto_stats)); return 0; }
    """
    with tempfile.TemporaryDirectory() as d:
        c = Path(d) / "r.c"
        c.write_text(src)
        exe = Path(d) / "r"
        subprocess.run(["gcc", "-I", str(HEADER.parent), str(c), "-o", str(exe)], check=True)
        size, off_layout, off_ps = (int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True,
                                                                    text=True).stdout.split())
    assert size == C.sizeof(abi.Records)
    assert off_layout == abi.Records.layout.offset and off_ps == abi.Records.proto_stats.offset


def test_unpack_layers_export_equals_the_mirrors():
    """pcppx_unpack_layers (the C decoder of PCPPX_LAYOUT_PACKED) equals abi.unpack_layers on ragged chains, a
    partial last tile and chains longer than max_layers."""
    import numpy as np

    lib = abi.load_engine()
    rng = np.random.default_rng(7)
    for n, ml in ((1, 1), (63, 4), (64, 12), (200, 8), (1000, 12)):
        s = np.zeros(n, abi.SUMMARY_DTYPE)
        s["n_layers"] = rng.integers(0, 16, n)
        packed = np.zeros(max(n * ml, 1), abi.LAYER_DTYPE)
        packed["offset"] = rng.integers(0, 65535, len(packed))
        packed["proto"] = rng.integers(1, 40, len(packed))
        fixed = np.ones(n * ml, abi.LAYER_DTYPE)
        assert lib.pcppx_unpack_layers(s.ctypes.data, packed.ctypes.data, n, ml, fixed.ctypes.data) == 0
        want = abi.unpack_layers(s, packed, ml)
        got = fixed.reshape(n, ml)
        valid = np.arange(ml)[None, :] < np.minimum(s["n_layers"], ml)[:, None]
        for f in abi.LAYER_DTYPE.names:
            assert (got[f][valid] == want[f][valid]).all(), (n, ml, f)
            assert (got[f][~valid] == 0).all(), (n, ml, f)
    assert lib.pcppx_unpack_layers(None, None, 5, 4, None) == abi.E_INVAL
    assert lib.pcppx_unpack_layers(s.ctypes.data, packed.ctypes.data, n, abi.PACKED_MAX_LAYERS + 1,
                                   fixed.ctypes.data) == abi.E_INVAL


def test_consumers_refuse_packed_records_without_gpu():
    """pcppx_filter_device / pcppx_reasm_device read FIXED records: PACKED ones (records.layout, written by the parse)
    are refused with PCPPX_E_INVAL before any device work."""
    lib = abi.load_engine()
    b = abi.Batch(1, 1, 1, 1, 1, 1, 0)
    r = abi.Records(1, 1)
    r.layout = abi.LAYOUT_PACKED
    spec = abi.MatchSpec()
    ctx = C.c_void_p(1)  # never dereferenced: the argument checks fail first
    assert lib.pcppx_reasm_device(ctx, C.byref(b), C.byref(r), 8, C.c_void_p(1), None) == abi.E_INVAL
    assert lib.pcppx_filter_device(ctx, C.byref(b), C.byref(r), 8, C.byref(spec), 0, C.c_void_p(1), C.c_void_p(1),
                                   1024, C.c_void_p(1), C.c_void_p(1), None) == abi.E_INVAL
