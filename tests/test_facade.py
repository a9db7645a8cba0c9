"""The facade's per-packet entry points (include/pcppx.hpp): PcapFileReaderDevice::getNextPacket / receivePackets /
getNextPackets over the prefetching zero-copy page pipeline, and Packet(RawPacket*, ...) bound to GPU records.

CPU: the reader hands out exactly what the reference's PcapFileReaderDevice / PcapNgFileReaderDevice return from
getNextPacket (tests/golden/ingest/expected.npz: caplen, frame length, timestamp, link type and bytes of every packet
of 3,155 captures) in all three read modes; and the drop-in benchmark's packet loop is the reference's token for
token (Examples/PcapPlusPlus-benchmark/benchmark.cpp:89-95).

GPU: every Packet built from a reader's RawPacket -- Packet(&raw), Packet(&raw, TCP), Packet(&raw, IP),
Packet(&raw, OsiModelNetworkLayer), the 4-argument form, the options mixed packet by packet (pages re-parsed for
options other than the reader learnt), copies of a RawPacket, the caller's own bytes (one-packet batches) and
freeRawPacket -- equals the C restatement's records for the same options bit for bit; with the reference
registered as host parser, every packet equals the reference Packet++ (layers, hashes)."""
from __future__ import annotations

import re
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

import ingest_cases as ic
import oracle
from conftest import GOLDEN, ROOT, load_golden, make_examples
from pcapplusplus_amd import abi, synth
from pcapplusplus_amd.pcap import from_packets, write_pcap

BIN = ROOT / "examples" / "bin"
CHECK = BIN / "facade_check"
GOLD = GOLDEN / "ingest"
REF = Path("/root/reference")


@pytest.fixture(scope="module")
def built():
    r = make_examples()
    assert r.returncode == 0, r.stderr
    return CHECK


def _read_dump(path: Path):
    raw = path.read_bytes()
    if raw == b"NOOPEN":
        return None
    out = {"packets": [], "caplens": [], "frame_lens": [], "ts_ns": [], "linktypes": []}
    pos = 0
    while pos < len(raw):
        cap, flen, ts, lt = struct.unpack_from("<IIQI", raw, pos)
        pos += 20
        out["packets"].append(raw[pos:pos + cap])
        pos += cap
        out["caplens"].append(cap)
        out["frame_lens"].append(flen)
        out["ts_ns"].append(ts)
        out["linktypes"].append(lt)
    for k, t in (("caplens", np.uint32), ("frame_lens", np.uint32), ("ts_ns", np.uint64), ("linktypes", np.uint32)):
        out[k] = np.array(out[k], t)
    return out


@pytest.mark.parametrize("mode", ["packet", "burst:64", "batch:333", "vector", "vector:333"])
def test_reader_entry_points_equal_reference(built, tmp_path, mode):
    """getNextPacket(RawPacket&) / receivePackets(RawPacket**, 64) / getNextBatch(RawBatch&, 333) /
    getNextPackets(RawPacketVector&) (all at once, and 333 per call) over every fixture, crafted case and mutation of the
    ingest golden set: the reference readers' packets, field for field."""
    from test_ingest import _case_bytes, _golden

    g, starts = _golden()
    data = _case_bytes(g)
    names, files = [], []
    for k, name in enumerate(g["names"]):
        b = data[str(name)]
        if b is None:
            continue
        f = tmp_path / f"c{k}"
        f.write_bytes(b)
        names.append(k)
        files.append(str(f))
    out = tmp_path / "out"
    out.mkdir()
    for lo in range(0, len(files), 400):  # argv length
        r = subprocess.run([str(built), "read", mode, str(out), *files[lo:lo + 400]], capture_output=True, text=True,
                           timeout=600)
        assert r.returncode == 0, r.stderr
        for j in range(lo, min(lo + 400, len(files))):
            (out / f"{j - lo}.bin").rename(out / f"r{j}.bin")
    checked = 0
    for j, k in enumerate(names):
        got = _read_dump(out / f"r{j}.bin")
        assert (got is not None) == bool(g["opened"][k]), f"{g['names'][k]}: open"
        if got is None:
            continue
        s, e = starts[k], starts[k + 1]
        assert len(got["caplens"]) == e - s, f"{g['names'][k]}: packet count {len(got['caplens'])} vs {e - s}"
        for key in ("caplens", "frame_lens", "ts_ns", "linktypes"):
            assert np.array_equal(got[key], g[key][s:e]), f"{g['names'][k]}: {key}"
        assert np.array_equal(ic.digest(got["packets"]), g["digests"][s:e]), f"{g['names'][k]}: packet bytes"
        checked += 1
    assert checked > 2500


def test_reader_pages_span_a_large_capture(built, tmp_path):
    """A capture larger than the first pages (16k, then 64k, 256k packets): getNextPacket crosses page boundaries
    with nothing lost or repeated, and stops cleanly at the end."""
    b = synth.config(3, 90_000)
    f = tmp_path / "in.pcap"
    write_pcap(f, b)
    out = tmp_path / "o"
    out.mkdir()
    r = subprocess.run([str(built), "read", "packet", str(out), str(f)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = _read_dump(out / "0.bin")
    assert np.array_equal(got["caplens"], b.caplens.astype(np.uint32))
    assert ic.digest(got["packets"]).tolist() == ic.digest([b.packet(i) for i in range(b.n)]).tolist()


def test_benchmark_packet_loop_is_the_references():
    """examples/benchmark.cpp's packet branch is Examples/PcapPlusPlus-benchmark/benchmark.cpp:89-95 token for token
    (read from the reference where it is present; the namespace alias `pcpp = pcppx` aside)."""
    ref = REF / "Examples" / "PcapPlusPlus-benchmark" / "benchmark.cpp"
    if not ref.exists():
        pytest.skip("/root/reference absent")
    tok = lambda s: re.findall(r"[A-Za-z_][A-Za-z_0-9]*|::|->|[^\s\w]", s)  # noqa: E731
    want = tok("".join(ref.read_text().splitlines(keepends=True)[88:95]))
    ours = tok((ROOT / "examples" / "benchmark.cpp").read_text())
    assert want[:4] == ["start", "=", "std", "::"] and "getNextPacket" in want and "TCP" in want
    assert any(ours[i:i + len(want)] == want for i in range(len(ours))), "packet loop differs from the reference's"
    # FilterTraffic's burst loop body: `pcpp::Packet parsedPacket(packetArr[i]);` and the flow-table lines
    ft = tok((ROOT / "examples" / "filter_traffic.cpp").read_text())
    for line in ("pcpp::Packet parsedPacket(packetArr[i]);", "uint32_t hash = pcpp::hash5Tuple(&parsedPacket);",
                 "m_Stats.collectStats(parsedPacket);", "pcapWriter->writePacket(*packetArr[i]);"):
        w = tok(line)
        assert any(ft[i:i + len(w)] == w for i in range(len(ft))), line


def test_benchmark_google_loops_are_the_references():
    """examples/benchmark_google_loops.inc holds BM_FileRead, BM_PacketParsing and BM_PacketPureParsing of
    Examples/PcapPlusPlus-benchmark/benchmark-google.cpp:15-64,149-207,209-264 token for token (signature and body;
    comments aside): the parse loops of the reference's third caller compile unchanged against the facade
    (examples/benchmark_google.cpp, `namespace pcpp = pcppx`) and against the reference (oracle/ref_benchmark_google.cpp)."""
    ref = REF / "Examples" / "PcapPlusPlus-benchmark" / "benchmark-google.cpp"
    if not ref.exists():
        pytest.skip("/root/reference absent")
    strip = lambda s: re.sub(r"//[^\n]*", "", s)  # noqa: E731
    tok = lambda s: re.findall(r"[A-Za-z_][A-Za-z_0-9]*|::|->|\"(?:[^\"\\]|\\.)*\"|[^\s\w]", strip(s))  # noqa: E731
    lines = ref.read_text().splitlines(keepends=True)
    ours = tok((ROOT / "examples" / "benchmark_google_loops.inc").read_text())
    for lo, hi, name in ((15, 64, "BM_FileRead"), (149, 207, "BM_PacketParsing"), (209, 264, "BM_PacketPureParsing")):
        want = tok("".join(lines[lo - 1:hi]))
        assert want[:4] == ["static", "void", name, "("] and want[-1] == "}", name
        assert any(ours[i:i + len(want)] == want for i in range(len(ours))), f"{name} differs from the reference's"
    # both programs include the same loops; the engine's aliases the namespace and nothing else
    eng = (ROOT / "examples" / "benchmark_google.cpp").read_text()
    assert '#include "benchmark_google_loops.inc"' in eng and "namespace pcpp = pcppx;" in eng
    assert '#include "../examples/benchmark_google_loops.inc"' in (ROOT / "oracle" / "ref_benchmark_google.cpp").read_text()


def test_create_reader_by_content(built, tmp_path):
    """IFileReaderDevice::createReader / tryCreateReader (PcapFileDevice.cpp:546-596) pick the reader from the first
    bytes: pcap (micro / nano, either byte order) and pcapng open; zstd, snoop, Kuznetzov-modified pcap, short and
    missing files give nullptr (tryCreateReader), as in the reference built without zstd and (here) without snoop."""
    b = synth.config(2, 10)
    good = tmp_path / "a.pcap"
    write_pcap(good, b)
    raw = good.read_bytes()
    cases = {"pcap": (raw, 10), "pcap_renamed.pcapng": (raw, 10),
             "nano.pcap": (bytes.fromhex("4d3cb2a1") + raw[4:], 10),
             "zstd.pcapng": (bytes.fromhex("28b52ffd") + raw[4:], None),
             "kuz.pcap": (bytes.fromhex("34cdb2a1") + raw[4:], None),
             "snoop": (b"snoop\0\0\0" + raw[8:], None), "short": (b"\xd4\xc3", None)}
    import os
    for name, (content, want) in cases.items():
        f = tmp_path / name
        f.write_bytes(content)
        r = subprocess.run([str(built), "create", str(f)], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        got = r.stdout.strip()
        assert got == ("null" if want is None else f"packets {want}"), (name, got)
    r = subprocess.run([str(built), "create", str(tmp_path / "missing.pcap")], capture_output=True, text=True, timeout=60)
    assert r.stdout.strip() == "null" and "Could not open file" in r.stderr
    assert os.path.exists(good)


# ---- GPU: Packet(RawPacket*, ...) records ----

VARIANTS = {  # facade_check plan name -> (parse_until_family, parse_until_osi)
    "full": (0, 8), "tcp": (4, 8), "ip": (0x203, 8), "osi2": (0, 2), "osi3": (0, 3), "osi4": (0, 4), "own": (0, 8),
    "copy": (4, 8),
    "free": (0, 8),
}
REC = np.dtype([("sum", abi.SUMMARY_DTYPE), ("lay", abi.LAYER_DTYPE, (abi.MAX_LAYERS,))])


def _env(host_parser=False, checksums=False):
    import os

    env = dict(os.environ)
    if host_parser:
        env["PCPPX_CHECK_HOST_PARSER"] = str(oracle.REF_SO)
    if checksums:
        env["PCPPX_CHECK_PAGE_CHECKSUMS"] = "1"
    return env


def _run_plan(built, tmp_path, batch, plan, host_parser=False, checksums=False):
    f, o = tmp_path / "in.pcap", tmp_path / "rec.bin"
    write_pcap(f, batch)
    env = _env(host_parser, checksums)
    r = subprocess.run([str(built), "parse", str(f), str(o), plan], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stderr
    rec = np.frombuffer(o.read_bytes(), REC)
    assert len(rec) == batch.n
    return rec


def _expected(batch, plan, reference=False, checksums=False):
    """per packet the records of the variant the plan applies to it: from the restatement (or the reference). The
    per-packet entry points compute no checksum (as Packet(&raw) in Packet++) unless setPageChecksums is on."""
    names = plan.split(",")
    want_sum = np.zeros(batch.n, abi.SUMMARY_DTYPE)
    want_lay = np.zeros((batch.n, abi.MAX_LAYERS), abi.LAYER_DTYPE)
    for v in set(names):
        fam, osi = VARIANTS[v]
        opts = abi.make_opts(fam, osi, checksums, abi.MAX_LAYERS)
        s, lay = oracle.ref_parse(batch, opts) if reference else oracle.oracle_parse(batch, opts, threads=8)
        idx = np.array([i for i in range(batch.n) if names[i % len(names)] == v], np.int64)
        want_sum[idx] = s[idx]
        want_lay[idx] = lay[idx]
    return want_sum, want_lay


def _captures():
    b, _ = load_golden(GOLDEN / "capture_example.npz")
    out = [("example.pcap", b)]
    for gname in ("pcap_lt1.npz", "pcap_lt113.npz", "pcap_lt276.npz", "pcap_lt0.npz", "dat_ethernet.npz"):
        gb, _ = load_golden(GOLDEN / gname)
        out.append((gname, gb))
    out.append(("synth_cfg5_40k", synth.config(5, 40_000)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("plan,checksums", [("full", False), ("tcp", False), ("osi3", False),
                                            ("full,tcp,ip,osi3,osi4", False), ("copy,free,tcp", False),
                                            ("full", True), ("full,tcp,copy", True)])
def test_gpu_packet_from_reader_equals_restatement(built, tmp_path, plan, checksums):
    """Every Packet a reader's RawPacket builds equals the restatement's records for its options, bit for bit
    (flagged packets: their exact prefix, as the device writes it); mixed plans force page re-parses. Pages hold the
    16-B brief + the chains (DENSE) and Packet::summary() rebuilds the protocol mask from the chain; with
    setPageChecksums the 32-B summaries with the checksum values."""
    for name, b in _captures():
        rec = _run_plan(built, tmp_path, b, plan, checksums=checksums)
        ws, wl = _expected(b, plan, checksums=checksums)
        try:
            oracle.compare_exact(rec["sum"], rec["lay"], ws, wl)
        except AssertionError as e:
            raise AssertionError(f"{name}: {e}") from None


@pytest.mark.gpu
def test_gpu_packet_from_own_bytes(built, tmp_path):
    """A RawPacket over the caller's own bytes (not from a reader) is parsed as a one-packet batch: the same records."""
    b, _ = load_golden(GOLDEN / "capture_example.npz")
    b = b.slice(0, 1500)
    rec = _run_plan(built, tmp_path, b, "own,full")
    ws, wl = _expected(b, "own,full")
    oracle.compare_exact(rec["sum"], rec["lay"], ws, wl)


def _run_vec(built, tmp_path, batch, plan, how, host_parser=False):
    f, o = tmp_path / "in.pcap", tmp_path / "rec.bin"
    write_pcap(f, batch)
    env = _env(host_parser)
    r = subprocess.run([str(built), "parsevec", str(f), str(o), plan, how], capture_output=True, text=True, timeout=600,
                       env=env or _env())
    assert r.returncode == 0, r.stderr
    import json

    info = json.loads(r.stdout.strip().splitlines()[-1])
    rec = np.frombuffer(o.read_bytes(), REC)
    assert len(rec) == batch.n == info["packets"]
    return rec, info


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["reader", "own", "copy"])
def test_gpu_packet_vector_equals_restatement(built, tmp_path, how):
    """benchmark-google.cpp's preload-then-parse pattern (:231-260): getNextPackets(RawPacketVector&) into page-bound
    RawPackets (reader), the caller's own RawPackets in a RawPacketVector (own: parsed together on the first Packet,
    one GPU batch per link type and options -- never one per packet), and a deep copy of the reader's vector (copy:
    bytes and records copied, no page kept); every Packet(vector.at(i), ...) equals the restatement's records."""
    for plan in ("full", "full,tcp,osi3"):
        for name, b in _captures():
            rec, info = _run_vec(built, tmp_path, b, plan, how)
            ws, wl = _expected(b, plan)
            try:
                oracle.compare_exact(rec["sum"], rec["lay"], ws, wl)
            except AssertionError as e:
                raise AssertionError(f"{name}/{plan}/{how}: {e}") from None
            # a parse per page (or group) and option set, plus at most one small parse of its chains deeper than the
            # records hold (their complete records, Records::side)
            variants = len(set(plan.split(",")))
            if how == "own":  # one group (one link type) parsed once per option set
                assert variants <= info["gpu_parses"] <= 2 * variants, (name, plan, info)
            else:  # pages of 16k (1k from 32 MiB of file on), then x4 up to 1M packets: each parsed once per option set
                fbytes = 24 + 16 * b.n + int(np.asarray(b.caplens, dtype=np.int64).sum())  # (plus copies' groups)
                pages, size, left = 0, (1024 if fbytes >= 32 << 20 else 16384), b.n
                while left > 0:
                    pages, left, size = pages + 1, left - size, min(size * 4, 1 << 20)
                pages = max(pages, 1) + (how == "copy")
                assert info["gpu_parses"] <= 2 * pages * variants, (name, plan, info)


@pytest.mark.gpu
def test_gpu_packet_vector_host_parser_equals_reference(built, tmp_path):
    """The caller's own RawPacketVector with the reference registered as host parser: every Packet equals the reference
    Packet++'s chain and hashes (flagged packets completed on the host)."""
    if not oracle.ref_available():
        pytest.skip("reference library not built")
    for name, b in _captures()[:-1]:
        rec, _ = _run_vec(built, tmp_path, b, "full", "own", host_parser=True)
        ws, wl = _expected(b, "full", reference=True)
        nl = np.minimum(ws["n_layers"], abi.MAX_LAYERS)
        for f in ("hash5", "hash5_dir", "hash2"):
            assert np.array_equal(rec["sum"][f], ws[f]), f"{name}: {f}"
        assert np.array_equal(rec["sum"]["n_layers"], nl), name
        valid = np.arange(abi.MAX_LAYERS)[None, :] < nl[:, None]
        for f in ("proto", "offset", "hdr_len", "data_len"):
            assert not ((rec["lay"][f] != wl[f]) & valid).any(), f"{name}: layers.{f}"


@pytest.mark.gpu
def test_gpu_copied_rawpackets_keep_no_page(built, tmp_path):
    """A copy of a reader's RawPacket owns its bytes and its records (RawPacket.cpp copyDataFrom), not the page: after the
    reader is closed, RawPackets kept from every page hold no page-locked record memory, and Packets built
    on them afterwards carry the same hashes as the restatement."""
    import json

    b = synth.config(3, 350_000)
    f = tmp_path / "in.pcap"
    write_pcap(f, b)
    r = subprocess.run([str(built), "retain", str(f), "997"], capture_output=True, text=True, timeout=600, env=_env())
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["kept"] == (b.n + 996) // 997 and d["pinned_while_reading"] > 0 and d["pinned_after"] == 0, d
    s, _ = oracle.oracle_parse(b, abi.make_opts(0, 8, False, 0), threads=8)
    assert d["h"] == int(s["hash5"][::997].astype(np.uint64).sum())


@pytest.mark.gpu
def test_gpu_packet_large_capture_pages(built, tmp_path):
    """350k IMIX packets (pages of 16k, 64k, 256k packets, parsed ahead by the pipeline) under Packet(&raw, TCP):
    every record equal to the restatement's."""
    b = synth.config(3, 350_000)
    rec = _run_plan(built, tmp_path, b, "tcp")
    ws, wl = _expected(b, "tcp")
    oracle.compare_exact(rec["sum"], rec["lay"], ws, wl)


@pytest.mark.gpu
@pytest.mark.parametrize("plan", ["full", "tcp", "full,tcp,osi3"])
def test_gpu_packet_host_parser_equals_reference(built, tmp_path, plan):
    """With the reference registered as host parser (setHostParser), every Packet -- flagged ones completed on the
    host -- equals the reference Packet++'s chain and hashes for its options."""
    if not oracle.ref_available():
        pytest.skip("reference library not built")
    for name, b in _captures()[:-1]:
        rec = _run_plan(built, tmp_path, b, plan, host_parser=True)
        ws, wl = _expected(b, plan, reference=True)
        s = rec["sum"]
        nl = np.minimum(ws["n_layers"], abi.MAX_LAYERS)
        for f in ("hash5", "hash5_dir", "hash2"):
            bad = np.nonzero(s[f] != ws[f])[0]
            assert len(bad) == 0, f"{name}: {f} differs on {len(bad)}; first {bad[:3]}"
        bad = np.nonzero(s["n_layers"] != nl)[0]
        assert len(bad) == 0, f"{name}: n_layers differs on {len(bad)}; first {bad[:3]}"
        valid = np.arange(abi.MAX_LAYERS)[None, :] < nl[:, None]
        for f in ("proto", "offset", "hdr_len", "data_len"):
            bad = np.nonzero(((rec["lay"][f] != wl[f]) & valid).any(axis=1))[0]
            assert len(bad) == 0, f"{name}: layers.{f} differs on {len(bad)}; first {bad[:3]}"


GOLDEN_PLAN = {"full": "full", "until_tcp": "tcp", "until_ip": "ip", "until_osi3": "osi3", "until_osi2": "osi2"}
CSUM_FLAGS = abi.F_IP_CSUM | abi.F_IP_CSUM_OK | abi.F_L4_CSUM | abi.F_L4_CSUM_OK


@pytest.mark.gpu
def test_gpu_host_completion_every_golden_record(built, tmp_path):
    """Every golden set under every parse-option variant, read through the facade (getNextPacket + Packet(&raw, ...))
    with the reference registered as host parser: every record -- the packets the engine finishes itself and the
    flagged ones the host parser completes (their hashes, port layer, protocol mask and checksums included) -- equals
    the reference Packet++'s golden record, field for field (flags: the reference's, plus F_HOST_PARSED on the
    completed ones).
    The host parser completes exactly the packets the engine leaves to the host -- the restatement's NEEDS_HOST flags,
    packet for packet -- so the completed records (the reference compared with itself: they test the facade's side
    table, not the GPU) are kept apart from the engine-finished ones, which are the GPU evidence; both counts are the
    fixtures' exact counts."""
    if not oracle.ref_available():
        pytest.skip("reference library not built")
    from conftest import golden_files

    from pcapplusplus_amd.engine import PcapReader

    checked = completed = 0
    for path in golden_files():
        b, variants = load_golden(path)
        f = tmp_path / "lt.pcap"
        write_pcap(f, b.slice(0, 1))
        with PcapReader(f) as r:
            lt = r.linktype
        if lt != b.linktype:
            continue  # a link-type value no capture file carries through the readers (the reference's map it to invalid)
        for v, (opts, rs, rl) in variants.items():
            if v not in GOLDEN_PLAN:
                continue
            rec = _run_plan(built, tmp_path, b, GOLDEN_PLAN[v], host_parser=True, checksums=bool(opts.want_checksums))
            s, lay = rec["sum"], rec["lay"]
            ml = int(opts.max_layers)
            host = (s["flags"] & F_HOST) != 0
            # the packets the engine leaves to the host (the restatement's flags under the same options)
            o16 = abi.Opts.from_buffer_copy(opts)
            o16.max_layers = abi.MAX_LAYERS
            os_, _ = oracle.oracle_parse(b, o16, threads=8)
            left = ((os_["flags"] & abi.F_NEEDS_HOST) != 0) & ((os_["flags"] & abi.F_BAD_DESC) == 0)
            assert (host == left).all(), f"{path.name}/{v}: host-completed packets differ from the engine's flagged ones " \
                                         f"at {np.nonzero(host != left)[0][:5]}"
            csum = bool(opts.want_checksums)
            nl = np.minimum(s["n_layers"], ml)
            where = f"{path.name}/{v}"
            assert (nl == rs["n_layers"]).all(), f"{where}: n_layers {np.nonzero(nl != rs['n_layers'])[0][:5]}"
            fields = ["hash5", "hash5_dir", "hash2", "l4_layer", "proto_mask"]
            if csum:
                fields += ["ip_csum_calc", "ip_csum_stored", "l4_csum_calc", "l4_csum_stored"]
            for f in fields:
                bad = np.nonzero(s[f] != rs[f])[0]
                assert len(bad) == 0, f"{where}: {f} differs on {len(bad)} packets, first #{bad[0]} " \
                                      f"(host-completed: {bool(host[bad[0]])})"
            keep = ~np.uint16(F_HOST | (0 if csum else CSUM_FLAGS))
            fl = s["flags"] & keep
            if ml < abi.MAX_LAYERS:  # the reference record's depth cap is the variant's
                fl = (fl & ~np.uint16(abi.F_DEPTH_OVERFLOW)) | np.where(s["n_layers"] > ml, abi.F_DEPTH_OVERFLOW, 0)
            bad = np.nonzero(fl != (rs["flags"] & keep))[0]
            assert len(bad) == 0, f"{where}: flags differ on {len(bad)} packets, first #{bad[0]}: {s[bad[0]]} vs {rs[bad[0]]}"
            assert not (s["flags"] & abi.F_NEEDS_HOST).any(), f"{where}: a packet left uncompleted"
            valid = np.arange(ml)[None, :] < nl[:, None]
            for f in ("proto", "osi", "offset", "hdr_len", "data_len"):
                bad = np.nonzero(((lay[:, :ml][f] != rl[f]) & valid).any(axis=1))[0]
                assert len(bad) == 0, f"{where}: layers.{f} differs on {len(bad)} packets, first #{bad[0]}"
            checked += b.n
            completed += int(host.sum())
    # the fixtures' exact counts: 75,357 records the engine finishes on the GPU + 778 the host parser completes (round 6:
    # the 20 Cisco HDLC / NFLOG fixture records are the engine's now)
    assert (checked - completed, completed) == (75_357, 778), (checked, completed)


F_HOST = 0x4000  # pcppx::F_HOST_PARSED (include/pcppx.hpp)
