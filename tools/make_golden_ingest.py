"""Freeze the ingest parity fixtures under tests/golden/ingest/ (run in this container only).

Expected outputs come from the REAL reference readers — PcapFileReaderDevice / PcapNgFileReaderDevice over
LightPcapNg (Pcap++/src/PcapFileDevice.cpp, 3rdParty/LightPcapNg), compiled from /root/reference sources by
oracle/Makefile into oracle/_ref/libpcpp_ref.so and driven by oracle/ref_ingest.cpp (getNextPacket per
packet). Inputs:
  * every capture the reference's own tests hold (Tests/**/*.pcap|*.pcapng|*.cap) and the 53 fuzz
    regression samples (Tests/Fuzzers/RegressionTests/regression_samples); those up to 32 KiB are copied
    into tests/golden/ingest/files/ (data files of the reference's tests), the larger ones are re-read from
    /root/reference where it exists;
  * the crafted pcap / pcapng cases of tests/ingest_cases.py (seeded);
  * seeded mutations of the crafted cases and of the copied pcapng fixtures.
Each reference read runs in a child process (a malformed file may crash it); cases where the reference's
reading is undefined behaviour (ingest_cases.reference_undefined) are listed with the reason, not frozen.

  python tools/make_golden_ingest.py
Writes tests/golden/ingest/expected.npz and tests/golden/ingest/files/*.
"""
from __future__ import annotations

import hashlib
import json
import multiprocessing as mp
import shutil
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import ingest_cases as ic  # noqa: E402
import oracle  # noqa: E402

REF = Path("/root/reference")
OUT = ROOT / "tests" / "golden" / "ingest"
COPY_LIMIT = 32 * 1024
MUTATIONS_PER_SEED = 20


def reference_captures() -> list[Path]:
    t = REF / "Tests"
    files = [p for ext in ("*.pcap", "*.pcapng", "*.cap") for p in t.rglob(ext)]
    files += sorted((t / "Fuzzers" / "RegressionTests" / "regression_samples").iterdir())
    return sorted(set(files))


def flat(p: Path) -> str:
    return str(p.relative_to(REF)).replace("/", "__")


def _child(path: str, q) -> None:
    q.put(oracle.ref_read_capture(path))


def ref_read_safe(path: Path):
    """The reference reader's output, or the string 'crash' if its process died."""
    q = mp.Queue()
    pr = mp.Process(target=_child, args=(str(path), q))
    pr.start()
    try:
        r = q.get(timeout=60)
    except Exception:
        r = "crash"
    pr.join(10)
    if pr.exitcode not in (0, None):
        return "crash"
    return r


def packets_of(r: dict) -> list[bytes]:
    out, o = [], 0
    d = r["data"].tobytes()
    for c in r["caplens"]:
        out.append(d[o:o + int(c)])
        o += int(c)
    return out


def main() -> None:
    if not oracle.ref_available():
        raise SystemExit("oracle/_ref/libpcpp_ref.so missing: make -C oracle ref")
    if OUT.exists():
        shutil.rmtree(OUT)
    (OUT / "files").mkdir(parents=True)

    cases: list[tuple[str, str, bytes | None, Path | None]] = []  # (name, kind, bytes, ref path)
    ng_seeds = []
    for p in reference_captures():
        b = p.read_bytes()
        if len(b) <= COPY_LIMIT:
            (OUT / "files" / flat(p)).write_bytes(b)
            cases.append((flat(p), "fixture", b, None))
            if b[:4] == b"\x0a\x0d\x0d\x0a":
                ng_seeds.append((flat(p), b))
        else:
            cases.append((flat(p), "fixture_ref", None, p))
    crafted = ic.crafted_cases()
    cases += [(n, "crafted", b, None) for n, b in crafted]
    cases += [(n, "mutation", b, None) for n, b in ic.mutation_cases(crafted + ng_seeds, MUTATIONS_PER_SEED)]

    names, kinds, sizes, shas, opened = [], [], [], [], []
    counts, caplens, frame_lens, ts, lts, digests = [], [], [], [], [], []
    skipped = {}
    tmp = Path(tempfile.mkdtemp())
    for name, kind, data, ref_path in cases:
        if data is None:
            data = ref_path.read_bytes()
            path = ref_path
        else:
            path = tmp / "case"
            path.write_bytes(data)
        why = ic.reference_undefined(data)
        if why:
            skipped[name] = why
            continue
        r = ref_read_safe(path)
        if r == "crash":
            skipped[name] = "reference reader crashed"
            continue
        names.append(name)
        kinds.append(kind)
        sizes.append(len(data))
        shas.append(hashlib.sha1(data).hexdigest())
        opened.append(r is not None)
        if r is None:
            counts.append(0)
            continue
        counts.append(len(r["caplens"]))
        caplens.append(r["caplens"])
        frame_lens.append(r["frame_lens"])
        ts.append(r["ts_ns"])
        lts.append(r["linktypes"])
        digests.append(ic.digest(packets_of(r)))
    cat = lambda xs, t: np.concatenate(xs).astype(t) if xs else np.zeros(0, t)  # noqa: E731
    np.savez_compressed(OUT / "expected.npz", names=np.array(names), kinds=np.array(kinds),
                        sizes=np.array(sizes, np.int64), sha1=np.array(shas), opened=np.array(opened),
                        counts=np.array(counts, np.int64), caplens=cat(caplens, np.uint32),
                        frame_lens=cat(frame_lens, np.uint32), ts_ns=cat(ts, np.uint64),
                        linktypes=cat(lts, np.uint32), digests=cat(digests, np.uint64),
                        mutations_per_seed=np.int64(MUTATIONS_PER_SEED),
                        ng_seed_names=np.array([n for n, _ in ng_seeds]),
                        skipped=np.array(json.dumps(skipped, sort_keys=True)))
    by_kind = {k: kinds.count(k) for k in sorted(set(kinds))}
    print(f"{len(names)} cases frozen {by_kind}, {sum(counts)} packets, {len(skipped)} skipped "
          f"({sorted(set(skipped.values()))})")


if __name__ == "__main__":
    main()
