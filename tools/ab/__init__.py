"""TOOLS ONLY: ctypes binding of tools/ab/libpcppx_ab.so — the A/B and diagnostic kernels (lane-per-packet
parse, tile-kernel shape variants, read-ceiling diagnostics, flow-table shapes) that were measured to pick the
product kernels. Never part of the product path (pcapplusplus_amd/ does not import this)."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

from pcapplusplus_amd import abi

AB_SO = Path(__file__).resolve().parent / "libpcppx_ab.so"
BASE_SO = Path(__file__).resolve().parent / "base" / "libpcppx_base.so"
_lib = None
_r01 = {}
BASE = -1  # parse_device variant: the final round-5 product kernel (tools/ab/base, commit afaa594, rebuilt from git)
BASE6_SO = Path(__file__).resolve().parent / "base" / "libpcppx_base6.so"
BASE6 = -2  # the round-6 kernel before the Cisco HDLC / NFLOG first layers (commit 1b98250, same recipe)

# pcppx_ab_parse_device variants (tools/ab/pcppx_ab.hip)
LANE, STREAM_ONLY, DIAG_TILE_READ, DIAG_GRID_READ = 1, 2, 3, 4  # (an unknown variant: PCPPX_E_INVAL)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not AB_SO.exists():
            raise RuntimeError(f"{AB_SO} missing: run `make -C tools/ab`")
        abi.load_engine()  # torch's HIP runtime first (one runtime per process)
        l = C.CDLL(str(AB_SO))
        P = C.c_void_p
        l.pcppx_ab_parse_device.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.Opts), C.POINTER(abi.Records), P, C.c_int]
        l.pcppx_ab_parse_device.restype = C.c_int
        l.pcppx_ab_flow_count_device.argtypes = [P, P, C.c_uint32, P, P, P, C.c_uint32, P, P, P, C.c_int, C.c_uint32]
        l.pcppx_ab_flow_count_device.restype = C.c_int
        l.pcppx_ab_flow_part.argtypes = [P, P, C.c_uint32, P, P, P, C.c_uint32, P, P, C.c_uint32, P, P, C.c_int]
        l.pcppx_ab_flow_part.restype = C.c_int
        _lib = l
    return _lib


def r01_lib(so: Path = BASE_SO) -> C.CDLL:
    """a product kernel rebuilt from git history (tools/ab/base)"""
    if so not in _r01:
        if not so.exists():
            raise RuntimeError(f"{so} missing: run `make -C {so.parent}`")
        abi.load_engine()
        l = C.CDLL(str(so))
        l.pcppx_r01_parse_device.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.Opts), C.POINTER(abi.Records), C.c_void_p]
        l.pcppx_r01_parse_device.restype = C.c_int
        _r01[so] = l
    return _r01[so]


def parse_device(data, offsets, caplens, n: int, linktype: int, opts: abi.Opts, summary, layers, stream: int,
                 variant: int, tuples=None, brief=None, flow_keys=None) -> None:
    b = abi.Batch(abi.ptr(data), abi.ptr(offsets), abi.ptr(caplens), int(data.numel()), n, linktype, 0)
    rec = abi.Records(abi.ptr(summary) if summary is not None else None,
                      abi.ptr(layers) if (layers is not None and opts.max_layers) else None, None,
                      abi.ptr(tuples) if tuples is not None else None)
    rec.brief = abi.ptr(brief) if brief is not None else None
    if flow_keys is not None:
        rec.flow_keys = abi.ptr(flow_keys)
    if variant in (BASE, BASE6):  # same opts / records layout (ABI 7)
        abi.check(r01_lib(BASE_SO if variant == BASE else BASE6_SO).pcppx_r01_parse_device(C.byref(b), C.byref(opts), C.byref(rec), C.c_void_p(stream or 0)),
                  "pcppx_r01_parse_device")
        return
    abi.check(lib().pcppx_ab_parse_device(C.byref(b), C.byref(opts), C.byref(rec), C.c_void_p(stream or 0), variant),
              "pcppx_ab_parse_device")


def parse_on_device(batch, opts: abi.Opts, variant: int, device: str = "cuda:0"):
    """parse_on_device through an A/B variant: (summary[n], layers[n, max_layers]) numpy records."""
    import torch

    from pcapplusplus_amd.engine import records_from_device, to_device

    data, offsets, caplens = to_device(batch, device)
    n = batch.n
    summary = torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device=device)
    layers = torch.zeros(max(n * opts.max_layers, 1) * 8, dtype=torch.uint8, device=device)
    parse_device(data, offsets, caplens, n, batch.linktype, opts, summary, layers,
                 torch.cuda.current_stream(device).cuda_stream, variant)
    torch.cuda.synchronize(device)
    return records_from_device(summary, layers, n, opts.max_layers)


def flow_count_device(summary, caplens, n: int, keys, packets, bytes_, capacity: int, stats, packed, stream: int,
                      shape: int, grid: int = 0) -> None:
    abi.check(lib().pcppx_ab_flow_count_device(abi.ptr(summary), abi.ptr(caplens), n, abi.ptr(keys), abi.ptr(packets),
                                               abi.ptr(bytes_), capacity, abi.ptr(stats),
                                               abi.ptr(packed) if packed is not None else None,
                                               C.c_void_p(stream or 0), shape, grid), "pcppx_ab_flow_count_device")
