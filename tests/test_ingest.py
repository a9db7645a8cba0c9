"""Native capture ingest (pcppx_pcap_*, csrc/pcppx_pcap.cpp) against the REAL reference readers.

tests/golden/ingest/expected.npz holds, per capture, what PcapFileReaderDevice / PcapNgFileReaderDevice
(Pcap++/src/PcapFileDevice.cpp over 3rdParty/LightPcapNg, compiled from the reference sources; generator
tools/make_golden_ingest.py) returned from getNextPacket: whether the device opened, and per packet the
caplen, frame length, timestamp (ns), link type and a BLAKE2b digest of the bytes. The captures are the
reference's own test captures and fuzz regression samples (copied under tests/golden/ingest/files/ up to
32 KiB; larger ones re-read from /root/reference when present), the crafted cases of ingest_cases.py and
their seeded mutations. Host only; the sanitizer test builds the reader with ASan/UBSan and replays
every fixture plus 200 mutations of each.
"""
from __future__ import annotations

import hashlib
import json
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import ingest_cases as ic

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden" / "ingest"
REF = Path("/root/reference")


def native_read_all(path, max_packets=777, data_cap=1 << 20):
    """Every packet through pcppx_pcap_read_batch_ex in batches of at most max_packets / data_cap bytes."""
    from pcapplusplus_amd.engine import PcapReader

    try:
        r = PcapReader(path)
    except RuntimeError:
        return None
    pk, cl, fl, ts, lt = [], [], [], [], []
    with r:
        while True:
            b = r.read_batch(max_packets, data_cap)
            if b.n == 0:
                break
            assert b.wire_bytes() <= data_cap and b.n <= max_packets
            pk += [b.packet(i) for i in range(b.n)]
            cl.append(b.caplens)
            fl.append(b.frame_lens)
            ts.append(b.timestamps_ns)
            lt += [b.linktype] * b.n
    cat = lambda xs, t: np.concatenate(xs).astype(t) if xs else np.zeros(0, t)  # noqa: E731
    return {"packets": pk, "caplens": cat(cl, np.uint32), "frame_lens": cat(fl, np.uint32),
            "ts_ns": cat(ts, np.uint64), "linktypes": np.array(lt, np.uint32)}


def native_map_all(path, max_packets=777):
    """Every packet through the zero-copy pcppx_pcap_map_batch (the bytes read out of the reader's map)."""
    import ctypes as C

    from pcapplusplus_amd.engine import PcapReader

    try:
        r = PcapReader(path)
    except RuntimeError:
        return None
    pk, cl, fl, ts, lt = [], [], [], [], []
    with r:
        while True:
            base, size, off, cap, flen, t = r.map_batch(max_packets)
            if len(cap) == 0:
                break
            assert len(cap) <= max_packets and (off + cap <= size).all()
            assert (np.diff(off.astype(np.int64)) > 0).all()  # ascending: the host path stages near-contiguous runs
            pk += [C.string_at(base + int(o), int(c)) for o, c in zip(off, cap)]
            cl.append(cap)
            fl.append(flen)
            ts.append(t)
            lt += [r.linktype] * len(cap)
    cat = lambda xs, t: np.concatenate(xs).astype(t) if xs else np.zeros(0, t)  # noqa: E731
    return {"packets": pk, "caplens": cat(cl, np.uint32), "frame_lens": cat(fl, np.uint32),
            "ts_ns": cat(ts, np.uint64), "linktypes": np.array(lt, np.uint32)}


def _golden():
    g = np.load(GOLD / "expected.npz")
    starts = np.concatenate([[0], np.cumsum(g["counts"])])
    return g, starts


def _case_bytes(g) -> dict[str, bytes | None]:
    """name -> capture bytes, rebuilt exactly as the generator made them (None: needs /root/reference)."""
    out = {}
    crafted = ic.crafted_cases()
    seeds = [(str(n), (GOLD / "files" / str(n)).read_bytes()) for n in g["ng_seed_names"]]
    for name, data in crafted + ic.mutation_cases(crafted + seeds, int(g["mutations_per_seed"])):
        out[name] = data
    for name, kind in zip(g["names"], g["kinds"]):
        name = str(name)
        if kind == "fixture":
            out[name] = (GOLD / "files" / name).read_bytes()
        elif kind == "fixture_ref":
            p = REF / name.replace("__", "/")
            out[name] = p.read_bytes() if p.exists() else None
    return out


def test_golden_covers_the_reference_fixtures():
    g, _ = _golden()
    kinds = list(g["kinds"])
    assert kinds.count("fixture") + kinds.count("fixture_ref") >= 220   # Tests/** captures + 53 fuzz samples
    assert kinds.count("crafted") >= 100 and kinds.count("mutation") >= 2000
    assert int(g["counts"].sum()) > 40000
    skipped = json.loads(str(g["skipped"]))
    assert set(skipped.values()) <= {"block total length below 12", "short interface block",
                                     "short enhanced packet block", "short simple packet block",
                                     "simple packet block before any interface",
                                     "simple packet block original length beyond its body"}


@pytest.mark.parametrize("kind", ["fixture", "fixture_ref", "crafted", "mutation"])
def test_reader_equals_reference(tmp_path, kind):
    g, starts = _golden()
    data = _case_bytes(g)
    checked = 0
    for k, name in enumerate(g["names"]):
        if g["kinds"][k] != kind:
            continue
        name = str(name)
        b = data[name]
        if b is None:
            continue  # large reference capture, /root/reference absent
        assert hashlib.sha1(b).hexdigest() == str(g["sha1"][k]), f"{name}: input differs from the frozen one"
        f = tmp_path / "case"
        f.write_bytes(b)
        # vary the batch limits so batches split on count, buffer size and link-type changes
        got = native_read_all(f, max_packets=1 + (k * 37) % 300, data_cap=(1 << 20) if k % 3 else 70000)
        assert (got is not None) == bool(g["opened"][k]), f"{name}: open"
        if got is None:
            continue
        s, e = starts[k], starts[k + 1]
        assert len(got["caplens"]) == e - s, f"{name}: packet count {len(got['caplens'])} vs {e - s}"
        for key in ("caplens", "frame_lens", "ts_ns", "linktypes"):
            assert np.array_equal(got[key], g[key][s:e]), f"{name}: {key}"
        assert np.array_equal(ic.digest(got["packets"]), g["digests"][s:e]), f"{name}: packet bytes"
        checked += 1
    if kind != "fixture_ref":
        assert checked > 50
    elif checked == 0:
        pytest.skip("/root/reference absent: the large reference captures are checked where it exists")


@pytest.mark.parametrize("kind", ["fixture", "crafted", "mutation"])
def test_zero_copy_reader_equals_reference(tmp_path, kind):
    """pcppx_pcap_map_batch: the same packets, lengths, timestamps and link types as the reference readers, read in
    place from the memory-mapped capture."""
    g, starts = _golden()
    data = _case_bytes(g)
    checked = 0
    for k, name in enumerate(g["names"]):
        if g["kinds"][k] != kind:
            continue
        b = data[str(name)]
        f = tmp_path / "case"
        f.write_bytes(b)
        got = native_map_all(f, max_packets=1 + (k * 53) % 400)
        assert (got is not None) == bool(g["opened"][k]), f"{name}: open"
        if got is None:
            continue
        s, e = starts[k], starts[k + 1]
        assert len(got["caplens"]) == e - s, f"{name}: packet count"
        for key in ("caplens", "frame_lens", "ts_ns", "linktypes"):
            assert np.array_equal(got[key], g[key][s:e]), f"{name}: {key}"
        assert np.array_equal(ic.digest(got["packets"]), g["digests"][s:e]), f"{name}: packet bytes"
        checked += 1
    assert checked > 50


def test_reader_equals_live_reference_on_large_captures(tmp_path):
    """Where the compiled reference exists (this container), compare the large captures live too."""
    import oracle

    if not oracle.ref_available() or not REF.exists():
        pytest.skip("reference library or /root/reference absent")
    for p in [REF / "Tests/Pcap++Test/PcapExamples/example.pcap", REF / "Tests/Pcap++Test/PcapExamples/many_interfaces-1.pcapng",
              REF / "Tests/Pcap++Test/PcapExamples/pcapng-example.pcapng"]:
        want = oracle.ref_read_capture(p)
        got = native_read_all(p, max_packets=500)
        for key in ("caplens", "frame_lens", "ts_ns", "linktypes"):
            assert np.array_equal(got[key], want[key]), f"{p.name}: {key}"
        assert b"".join(got["packets"]) == want["data"].tobytes()


def test_pcapng_batches_hold_one_linktype(tmp_path):
    """Interfaces of different link types (Ethernet, Linux SLL, raw IP) interleaved packet by packet:
    every batch is uniform and the batches alternate."""
    from pcapplusplus_amd.engine import PcapReader

    f = tmp_path / "multi.pcapng"
    f.write_bytes(dict(ic.crafted_cases())["ng_multi_if"])
    seen = []
    with PcapReader(f) as r:
        while True:
            b = r.read_batch(1000, 1 << 20)
            if b.n == 0:
                break
            seen.append(b.linktype)
    assert len(set(seen)) > 1 and all(a != b for a, b in zip(seen, seen[1:]))


def test_buffer_limits(tmp_path):
    from pcapplusplus_amd.engine import PcapReader

    pk = ic.sample_packets(100)
    f = tmp_path / "buf.pcap"
    f.write_bytes(ic.pcap_file(pk))
    with PcapReader(f) as r:
        with pytest.raises(RuntimeError):
            r.read_batch(10, data_cap=16)  # one record does not fit: PCPPX_E_NOMEM, nothing consumed
        b = r.read_batch(10, data_cap=1 << 20)
        assert [b.packet(i) for i in range(b.n)] == pk[:10]
    with PcapReader(f) as r:
        b = r.read_batch(1000, data_cap=4096)
        assert 0 < b.n < 100 and b.wire_bytes() <= 4096
        assert [b.packet(i) for i in range(b.n)] == pk[:b.n]


def test_rejects_missing_and_unknown(tmp_path):
    from pcapplusplus_amd.engine import PcapReader

    with pytest.raises(RuntimeError):
        PcapReader(tmp_path / "missing.pcap")
    f = tmp_path / "x.snoop"
    f.write_bytes(b"snoop\0\0\0" + b"\0" * 60)  # snoop: a format the engine does not read
    with pytest.raises(RuntimeError):
        PcapReader(f)


def test_sanitizers(tmp_path):
    """pcppx_pcap.cpp under ASan + UBSan (host build, no HIP) over every fixture, crafted case and 200
    seeded mutations of each fixture (tools/ingest_fuzz.cpp)."""
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ absent")
    exe = tmp_path / "ingest_fuzz"
    subprocess.run([gxx, "-std=c++17", "-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    f"-I{ROOT / 'include'}", str(ROOT / "pcapplusplus_amd/csrc/pcppx_pcap.cpp"),
                    str(ROOT / "tools/ingest_fuzz.cpp"), "-o", str(exe)], check=True)
    cdir = tmp_path / "crafted"
    cdir.mkdir()
    for name, data in ic.crafted_cases():
        (cdir / name).write_bytes(data)
    files = sorted(str(p) for p in (GOLD / "files").iterdir()) + sorted(str(p) for p in cdir.iterdir())
    env = {"TMPDIR": str(tmp_path), "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([str(exe), "200"] + files, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.startswith(f"files={len(files)} ")


def _big_pcap(tmp_path, name, n, seed, zero_payload=False, snaplen=262144, corrupt_at=None, cut_tail=False):
    """A pcap large enough for the parallel record walk (>= 16 MiB), as bytes on disk."""
    import struct

    from pcapplusplus_amd import synth
    from pcapplusplus_amd.pcap import write_pcap

    b = synth.imix(n, seed)
    if zero_payload:  # runs of zero bytes parse as chains of empty records: the false-start hazard
        d = b.data.copy()
        for i in range(0, b.n, 3):
            o, c = int(b.offsets[i]), int(b.caplens[i])
            d[o + 54:o + c] = 0
        b = type(b)(d, b.offsets, b.caplens, b.linktype)
    f = tmp_path / name
    write_pcap(f, b, snaplen=snaplen)
    raw = bytearray(f.read_bytes())
    if corrupt_at is not None:  # an invalid record header: the stream ends there (readNextPacket, :799-886)
        pos = 24 + 16 * corrupt_at + int(b.caplens[:corrupt_at].sum())
        raw[pos + 8:pos + 12] = struct.pack("<I", 0x7FFFFFFF)
    if cut_tail:
        del raw[-37:]
    f.write_bytes(bytes(raw))
    return f


@pytest.mark.parametrize("case", ["clean", "zeros", "corrupt", "snaplen", "cut"])
def test_parallel_walk_equals_sequential(tmp_path, case):
    """pcppx_pcap_map_batch walks large pcap regions in parallel (re-synchronised segments merged where the chains
    meet): the same records as the sequential copying reader, on a 60-MiB capture -- clean, with runs of zero bytes
    that look like empty records, with an invalid record mid-file (the stream ends there), with a snapshot length
    below the packet sizes, and with the last record cut short."""
    import oracle

    if not oracle.ref_available():
        pytest.skip("the reference reader (oracle/_ref) is the sequential oracle here")
    kw = {"clean": {}, "zeros": {"zero_payload": True}, "corrupt": {"corrupt_at": 123_457},
          "snaplen": {"snaplen": 400}, "cut": {"cut_tail": True}}[case]
    f = _big_pcap(tmp_path, f"{case}.pcap", 180_000, 11, **kw)
    want = oracle.ref_read_capture(f)  # PcapFileReaderDevice::getNextPacket, one packet at a time
    cl = want["caplens"].astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(cl)])
    seq = {k: want[k] for k in ("caplens", "frame_lens", "ts_ns", "linktypes")}
    seq["packets"] = [want["data"][starts[i]:starts[i + 1]].tobytes() for i in range(len(cl))]
    par = native_map_all(f, max_packets=70_000)
    # the copying reader takes the parallel walk too: batches cut by the byte limit as well as the count
    cp = native_read_all(f, max_packets=50_000, data_cap=9_000_000)
    for key in ("caplens", "frame_lens", "ts_ns", "linktypes"):
        assert np.array_equal(cp[key], seq[key]), key
    assert cp["packets"] == seq["packets"]
    assert len(par["caplens"]) == len(seq["caplens"]) > 100_000 or case == "corrupt"
    for key in ("caplens", "frame_lens", "ts_ns", "linktypes"):
        assert np.array_equal(par[key], seq[key]), key
    assert par["packets"] == seq["packets"]
    if case == "corrupt":
        assert len(par["caplens"]) == 123_457


@pytest.mark.parametrize("cut", [False, True])
def test_parallel_walk_sanitized(tmp_path, cut):
    """The parallel record walk under AddressSanitizer / UBSan (host code only): a 60-MiB capture (clean, or with its
    last record cut short) read with three batch sizes, zero-copy and copying calls alternating on one reader -- the
    same packets and record checksum for every batch size, no sanitizer report."""
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ absent")
    exe = tmp_path / "ingest_parallel_check"
    subprocess.run([gxx, "-std=c++17", "-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    f"-I{ROOT / 'include'}", str(ROOT / "pcapplusplus_amd/csrc/pcppx_pcap.cpp"),
                    str(ROOT / "tools/ingest_parallel_check.cpp"), "-o", str(exe), "-lpthread"], check=True)
    f = _big_pcap(tmp_path, "big.pcap", 180_000, 5, cut_tail=cut)
    env = {"TMPDIR": str(tmp_path), "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([str(exe), str(f)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 3 and len({ln.split(": ", 1)[1] for ln in lines}) == 1, r.stdout
    assert int(lines[0].split(": ")[1].split()[0]) == (180_000 - 1 if cut else 180_000)
