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
    return stats


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
