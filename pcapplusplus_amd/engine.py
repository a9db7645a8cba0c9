"""Engine handle: one pcppx context (one GPU, one host thread) over the C ABI of include/pcppx.h.

Host batches (numpy) go through pcppx_parse_batch_host (pinned, double-buffered H2D -> kernel -> D2H);
device batches (torch tensors resident in HBM) through pcppx_parse_batch_device on a HIP stream.
There is no CPU fallback: a missing libpcppx.so or a missing GPU raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .pcap import PacketBatch


class Engine:
    def __init__(self, device: int = 0):
        self.lib = abi.load_engine()
        self.ctx = C.c_void_p()
        abi.check(self.lib.pcppx_open(device, C.byref(self.ctx)), "pcppx_open")
        self.device = device

    def close(self) -> None:
        if self.ctx:
            self.lib.pcppx_close(self.ctx)
            self.ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- host-resident batches ----
    def parse_host(self, batch: PacketBatch, opts: abi.Opts | None = None, out=None):
        """Parse a host batch; returns (summary[n], layers[n, max_layers]) numpy record arrays. out: caller-owned
        (summary, layers) arrays to fill (e.g. pinned_records(): the records then come back by DMA straight
        into them), else fresh zeroed arrays."""
        opts = opts or abi.make_opts()
        if out is None:
            summary = np.zeros(batch.n, dtype=abi.SUMMARY_DTYPE)
            layers = np.zeros(max(batch.n * opts.max_layers, 1), dtype=abi.LAYER_DTYPE)
        else:
            summary, layers = out
            if summary.shape[0] < batch.n or layers.size < batch.n * opts.max_layers:
                raise ValueError("output arrays too small for the batch")
        rec = abi.Records(summary.ctypes.data, layers.ctypes.data if opts.max_layers else None)
        b = batch.c_batch()
        abi.check(self.lib.pcppx_parse_batch_host(self.ctx, C.byref(b), C.byref(opts), C.byref(rec)),
                  "pcppx_parse_batch_host")
        return summary, layers[: batch.n * opts.max_layers].reshape(batch.n, opts.max_layers)

    def parse_host_ex(self, batch: PacketBatch, opts: abi.Opts, want_summary: bool = True, want_brief: bool = False,
                      pinned: bool = False):
        """Host parse with the ABI-7 outputs: the summary and / or the 16-B brief, and the layer entries in opts.layout
        (LAYOUT_FIXED: [n, max_layers]; LAYOUT_DENSE: the chains back to back, pcppx_records.layers_written of them).
        Returns (summary | None, brief | None, layers, layers_written). pinned: page-locked output arrays (records
        DMA'd straight into them)."""
        n, ml = batch.n, opts.max_layers
        keep = []

        def arr(count, dt):
            if not pinned:
                return np.zeros(count, dtype=dt)
            buf = PinnedBuffer(max(count, 1) * dt.itemsize)
            keep.append(buf)
            return buf.array.view(dt)[:count]

        summary = arr(n, abi.SUMMARY_DTYPE) if want_summary else None
        brief = arr(n, abi.BRIEF_DTYPE) if want_brief else None
        layers = arr(max(n * ml, 1), abi.LAYER_DTYPE)
        rec = abi.Records(summary.ctypes.data if summary is not None else None, layers.ctypes.data if ml else None)
        rec.brief = brief.ctypes.data if brief is not None else None
        b = batch.c_batch()
        abi.check(self.lib.pcppx_parse_batch_host(self.ctx, C.byref(b), C.byref(opts), C.byref(rec)),
                  "pcppx_parse_batch_host")
        w = int(rec.layers_written)
        out = (None if summary is None else summary.copy() if pinned else summary,
               None if brief is None else brief.copy() if pinned else brief,
               layers[:w].copy() if pinned else layers[:w], w)
        for k in keep:
            k.free()
        return out

    def window_choice(self, want_checksums: bool) -> int:
        """pcppx_window_choice: the window a WINDOW_DEFAULT launch would run with now (abi.WINDOW_*)."""
        w = C.c_int(0)
        abi.check(self.lib.pcppx_window_choice(self.ctx, 1 if want_checksums else 0, C.byref(w)), "pcppx_window_choice")
        return w.value

    # ---- device-resident batches (torch tensors on this GPU) ----
    def parse_device(self, data, offsets, caplens, n: int, linktype: int, opts: abi.Opts, summary, layers=None,
                     stream: int | None = None, flow_keys=None, tuples=None, proto_stats=None, brief=None) -> None:
        """Queue a parse of device tensors on `stream` (a hipStream_t handle, e.g.
        torch.cuda.current_stream().cuda_stream). summary: uint8 tensor of n*32 bytes (or None with no layers when
        tuples / flow_keys / proto_stats is given); layers: n*max_layers*8; flow_keys: n int32 (hash5); tuples: n*48
        bytes (5-tuple extracts); proto_stats: 16 x int64, accumulated (collectStats)."""
        b = abi.Batch(abi.ptr(data), abi.ptr(offsets), abi.ptr(caplens), int(data.numel()), n, linktype, 0)
        opt = lambda t: abi.ptr(t) if t is not None else None  # noqa: E731
        rec = abi.Records(opt(summary), abi.ptr(layers) if (layers is not None and opts.max_layers) else None,
                          opt(flow_keys), opt(tuples), opt(proto_stats))
        rec.brief = opt(brief)
        abi.check(self.lib.pcppx_parse_batch_device(self.ctx, C.byref(b), C.byref(opts), C.byref(rec),
                                                    C.c_void_p(stream or 0)), "pcppx_parse_batch_device")

    def flow_count_device(self, summary, caplens, n: int, keys, packets, bytes_, capacity: int, stats,
                          stream: int | None = None) -> None:
        abi.check(self.lib.pcppx_flow_count_device(self.ctx, abi.ptr(summary), abi.ptr(caplens), n, abi.ptr(keys),
                                                   abi.ptr(packets), abi.ptr(bytes_), capacity, abi.ptr(stats),
                                                   C.c_void_p(stream or 0)), "pcppx_flow_count_device")

    def flow_count_keys_device(self, flow_keys, caplens, n: int, keys, packets, bytes_, capacity: int, stats,
                               stream: int | None = None) -> None:
        """pcppx_flow_count_keys_device: the flow table over the dense hash5 column a parse wrote (flow_keys)."""
        abi.check(self.lib.pcppx_flow_count_keys_device(self.ctx, abi.ptr(flow_keys), abi.ptr(caplens), n, abi.ptr(keys),
                                                        abi.ptr(packets), abi.ptr(bytes_), capacity, abi.ptr(stats),
                                                        C.c_void_p(stream or 0)), "pcppx_flow_count_keys_device")

    def filter_device(self, data, offsets, caplens, n: int, linktype: int, summary, layers, max_layers: int,
                      spec: abi.MatchSpec, seq_base: int, flow_keys, flow_first, capacity: int, matched, stats,
                      stream: int | None = None) -> None:
        """FilterTraffic's worker over a parsed device batch (pcppx_filter_device). flow_keys/flow_first:
        zero-initialised u64 tensors of `capacity` (power of two) slots kept across batches; matched: u8[n];
        stats: 14 x u64 (abi.STATS_FIELDS order), accumulated."""
        b = abi.Batch(abi.ptr(data), abi.ptr(offsets), abi.ptr(caplens), int(data.numel()), n, linktype, 0)
        rec = abi.Records(abi.ptr(summary), abi.ptr(layers))
        abi.check(self.lib.pcppx_filter_device(self.ctx, C.byref(b), C.byref(rec), max_layers, C.byref(spec),
                                               seq_base, abi.ptr(flow_keys), abi.ptr(flow_first), capacity,
                                               abi.ptr(matched), abi.ptr(stats), C.c_void_p(stream or 0)),
                  "pcppx_filter_device")

    def reasm_device(self, data, offsets, caplens, n: int, linktype: int, summary, layers, max_layers: int, info,
                     stream: int | None = None) -> None:
        """The reassembly front ends (pcppx_reasm_device) over a parsed device batch: info is a uint8 tensor of
        n * 16 bytes (abi.REASM_DTYPE records)."""
        b = abi.Batch(abi.ptr(data), abi.ptr(offsets), abi.ptr(caplens), int(data.numel()), n, linktype, 0)
        rec = abi.Records(abi.ptr(summary), abi.ptr(layers))
        abi.check(self.lib.pcppx_reasm_device(self.ctx, C.byref(b), C.byref(rec), max_layers, abi.ptr(info),
                                              C.c_void_p(stream or 0)), "pcppx_reasm_device")

    def parse_reasm_device(self, data, offsets, caplens, n: int, linktype: int, opts: abi.Opts, summary, layers,
                           info, stream: int | None = None) -> None:
        """Parse + reassembly front ends in one kernel pass (pcppx_parse_batch_device_reasm)."""
        b = abi.Batch(abi.ptr(data), abi.ptr(offsets), abi.ptr(caplens), int(data.numel()), n, linktype, 0)
        rec = abi.Records(abi.ptr(summary), abi.ptr(layers))
        abi.check(self.lib.pcppx_parse_batch_device_reasm(self.ctx, C.byref(b), C.byref(opts), C.byref(rec),
                                                          abi.ptr(info), C.c_void_p(stream or 0)),
                  "pcppx_parse_batch_device_reasm")

    def filter_reset(self, capacity: int = 0) -> None:
        abi.check(self.lib.pcppx_filter_reset(self.ctx, capacity), "pcppx_filter_reset")

    def filter_host(self, batch: PacketBatch, spec: abi.MatchSpec):
        """FilterTraffic's worker over a host batch (context-held flow table): (matched u8[n], stats dict
        accumulated since the last filter_reset)."""
        matched = np.zeros(max(batch.n, 1), dtype=np.uint8)
        st = abi.PacketStats()
        b = batch.c_batch()
        abi.check(self.lib.pcppx_filter_batch_host(self.ctx, C.byref(b), C.byref(spec), matched.ctypes.data,
                                                   C.byref(st)), "pcppx_filter_batch_host")
        return matched[: batch.n], st.as_dict()

    def sync(self) -> None:
        abi.check(self.lib.pcppx_sync(self.ctx), "pcppx_sync")


class PcapReader:
    """Native capture ingest (pcppx_pcap_*): records of a pcap / pcapng capture copied straight into packed
    batches. Mirrors IFileReaderDevice (Pcap++/header/PcapFileDevice.h) open / getNextPackets / close; each
    batch carries one link type (RawPacket::getLinkLayerType), its timestamps and frame lengths."""

    def __init__(self, path: str, pinned: bool = False):
        self.lib = abi.load_engine()
        self.handle = C.c_void_p()
        abi.check(self.lib.pcppx_pcap_open(str(path).encode(), C.byref(self.handle)), f"pcppx_pcap_open({path})")
        self.linktype = int(self.lib.pcppx_pcap_linktype(self.handle))
        self.pinned = pinned

    def read_batch(self, max_packets: int = 1 << 20, data_cap: int = 256 << 20) -> PacketBatch:
        """Next batch of at most max_packets packets / data_cap bytes (n == 0 at end of file)."""
        data = np.empty(data_cap, dtype=np.uint8)
        offsets = np.empty(max_packets, dtype=np.uint64)
        caplens = np.empty(max_packets, dtype=np.uint32)
        frame_lens = np.empty(max_packets, dtype=np.uint32)
        ts = np.empty(max_packets, dtype=np.uint64)
        n, used = C.c_uint32(0), C.c_uint64(0)
        abi.check(self.lib.pcppx_pcap_read_batch_ex(self.handle, data.ctypes.data, data_cap, offsets.ctypes.data,
                                                    caplens.ctypes.data, frame_lens.ctypes.data, ts.ctypes.data,
                                                    max_packets, C.byref(n), C.byref(used)), "pcppx_pcap_read_batch_ex")
        k = n.value
        self.linktype = int(self.lib.pcppx_pcap_linktype(self.handle))
        return PacketBatch(data[: used.value].copy(), offsets[:k].copy(), caplens[:k].copy(), self.linktype,
                           timestamps_ns=ts[:k].copy(), frame_lens=frame_lens[:k].copy())

    def map_batch(self, max_packets: int = 1 << 20):
        """Zero-copy next batch (pcppx_pcap_map_batch): (map address, file size, offsets, caplens, frame_lens, ts);
        the bytes stay in the reader's memory map until close()."""
        offsets = np.empty(max_packets, dtype=np.uint64)
        caplens = np.empty(max_packets, dtype=np.uint32)
        frame_lens = np.empty(max_packets, dtype=np.uint32)
        ts = np.empty(max_packets, dtype=np.uint64)
        base, size, n = C.c_void_p(), C.c_uint64(0), C.c_uint32(0)
        abi.check(self.lib.pcppx_pcap_map_batch(self.handle, C.byref(base), C.byref(size), offsets.ctypes.data,
                                                caplens.ctypes.data, frame_lens.ctypes.data, ts.ctypes.data,
                                                max_packets, C.byref(n)), "pcppx_pcap_map_batch")
        k = n.value
        self.linktype = int(self.lib.pcppx_pcap_linktype(self.handle))
        return base.value, size.value, offsets[:k].copy(), caplens[:k].copy(), frame_lens[:k].copy(), ts[:k].copy()

    def close(self) -> None:
        if self.handle:
            self.lib.pcppx_pcap_close(self.handle)
            self.handle = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host memory (pcppx_host_alloc) viewed as a numpy uint8 array: a host batch whose bytes
    sit here is copied to HBM by DMA straight from it (no staging copy), as a NIC ring's buffers would be."""

    def __init__(self, nbytes: int):
        self.lib = abi.load_engine()
        self.ptr = self.lib.pcppx_host_alloc(max(1, nbytes))
        if not self.ptr:
            raise MemoryError(f"pcppx_host_alloc({nbytes}) failed")
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(1, nbytes)).from_address(self.ptr))

    def free(self) -> None:
        if self.ptr:
            self.array = None
            self.lib.pcppx_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def pinned_records(n: int, max_layers: int):
    """(summary[n], layers[n * max_layers]) record arrays in page-locked memory, plus the buffers to keep alive:
    pcppx_parse_batch_host then writes the records by DMA, with no host copy."""
    sb = PinnedBuffer(n * abi.SUMMARY_DTYPE.itemsize)
    lb = PinnedBuffer(max(1, n * max_layers) * abi.LAYER_DTYPE.itemsize)
    return (sb.array.view(abi.SUMMARY_DTYPE)[:n], lb.array.view(abi.LAYER_DTYPE)[: max(1, n * max_layers)]), (sb, lb)


def pinned_copy(batch: PacketBatch) -> tuple[PacketBatch, PinnedBuffer]:
    """The same batch with its bytes in page-locked memory (keep the buffer alive while the batch is used)."""
    buf = PinnedBuffer(batch.data.nbytes)
    buf.array[: batch.data.nbytes] = batch.data
    return PacketBatch(buf.array[: batch.data.nbytes], batch.offsets, batch.caplens, batch.linktype), buf


def device_count() -> int:
    n = C.c_int(0)
    abi.check(abi.load_engine().pcppx_device_count(C.byref(n)), "pcppx_device_count")
    return n.value


def to_device(batch: PacketBatch, device: str = "cuda:0"):
    """Copy a host batch into HBM as torch tensors: (data u8, offsets i64-as-u64, caplens i32-as-u32)."""
    import torch

    data = torch.from_numpy(batch.data).to(device)
    offsets = torch.from_numpy(batch.offsets.view(np.int64)).to(device)
    caplens = torch.from_numpy(batch.caplens.view(np.int32)).to(device)
    return data, offsets, caplens


def records_from_device(summary_t, layers_t, n: int, max_layers: int):
    s = summary_t.cpu().numpy().view(abi.SUMMARY_DTYPE)[:n]
    if layers_t is None or max_layers == 0:
        return s, np.zeros((n, 0), dtype=abi.LAYER_DTYPE)
    lay = layers_t.cpu().numpy().view(abi.LAYER_DTYPE)[: n * max_layers].reshape(n, max_layers)
    return s, lay


def parse_on_device_ex(eng: Engine, batch: PacketBatch, opts: abi.Opts | None = None, device: str = "cuda:0",
                       summary: bool = True, tuples: bool = False, proto_stats: bool = False, flow_keys: bool = False,
                       brief: bool = False):
    """parse_on_device with the optional outputs: {"summary", "brief" (16-B pcppx_brief), "layers" (FIXED
    [n, max_layers], decoded when the layout is PACKED, through the summary or else the brief), "packed" (the raw PACKED
    entries), "tuples", "proto_stats" (dict), "flow_keys" (u32 hash5)}."""
    import torch

    opts = opts or abi.make_opts()
    data, offsets, caplens = to_device(batch, device)
    n = batch.n
    st = torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device=device) if summary else None
    lay = torch.zeros(max(n * opts.max_layers, 1) * 8, dtype=torch.uint8, device=device)
    tp = torch.zeros(max(n, 1) * 48, dtype=torch.uint8, device=device) if tuples else None
    ps = torch.zeros(abi.PROTO_STATS, dtype=torch.int64, device=device) if proto_stats else None
    fk = torch.zeros(max(n, 1), dtype=torch.int32, device=device) if flow_keys else None
    br = torch.zeros(max(n, 1) * 16, dtype=torch.uint8, device=device) if brief else None
    eng.parse_device(data, offsets, caplens, n, batch.linktype, opts, st, lay if opts.max_layers else None,
                     torch.cuda.current_stream(device).cuda_stream, flow_keys=fk, tuples=tp, proto_stats=ps, brief=br)
    torch.cuda.synchronize(device)
    out = {}
    if st is not None:
        out["summary"] = st.cpu().numpy().view(abi.SUMMARY_DTYPE)[:n]
    if br is not None:
        out["brief"] = br.cpu().numpy().view(abi.BRIEF_DTYPE)[:n]
    if opts.max_layers and (st is not None or br is not None):
        raw = lay.cpu().numpy().view(abi.LAYER_DTYPE)[: n * opts.max_layers]
        if opts.layout == abi.LAYOUT_PACKED:
            out["packed"] = raw
            out["layers"] = abi.unpack_layers(out["summary"] if st is not None else out["brief"], raw, opts.max_layers)
        else:
            out["layers"] = raw.reshape(n, opts.max_layers)
    if tp is not None:
        out["tuples"] = tp.cpu().numpy().view(abi.TUPLE_DTYPE)[:n]
    if fk is not None:
        out["flow_keys"] = fk.cpu().numpy().view(np.uint32)[:n]
    if ps is not None:
        v = ps.cpu().numpy()
        out["proto_stats"] = {f: int(v[k]) for k, f in enumerate(abi.PROTO_STATS_FIELDS)}
        out["proto_stats_raw"] = v
    return out


def parse_on_device(eng: Engine, batch: PacketBatch, opts: abi.Opts | None = None, device: str = "cuda:0"):
    """Copy a host batch to HBM, run the device-resident parse, copy the records back."""
    import torch

    opts = opts or abi.make_opts()
    data, offsets, caplens = to_device(batch, device)
    n = batch.n
    summary = torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device=device)
    layers = torch.zeros(max(n * opts.max_layers, 1) * 8, dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    eng.parse_device(data, offsets, caplens, n, batch.linktype, opts, summary, layers, stream)
    torch.cuda.synchronize(device)
    return records_from_device(summary, layers, n, opts.max_layers)
