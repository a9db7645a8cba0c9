"""HBM traffic per launch of the parse kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py.

gfx950 correction (/opt/skills/guides/MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half of the
bytes of a wide (16 B/lane) coalesced streaming read; WRITE_SIZE is exact for 16-B-per-lane stores. Both
are in KiB. Our reads are dwordx4 (16 B/lane) loads, so hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024.
The result is keyed by everything bench.py checks before using it: config, packets, max_layers, checksums, layer
layout, record kind (taken from the bench line the profiled run printed) and the sha of the kernel source it was
measured on (bench.kernel_sha).

  python tools/pmc_traffic.py <fetch_dir> <write_dir> <bench line .json> <out.json>
"""
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import kernel_sha  # noqa: E402


def per_launch(d: str, counter: str) -> tuple[float, int]:
    vals = []
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "parse_tile_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows in {d}")
    vals.sort()
    return vals[len(vals) // 2], len(vals)  # median over launches


fetch_kib, nf = per_launch(sys.argv[1], "FETCH_SIZE")
write_kib, nw = per_launch(sys.argv[2], "WRITE_SIZE")
line = json.loads(Path(sys.argv[3]).read_text().strip().splitlines()[-1])
c = line["config"]
out = {
    "config": int(c["workload"].split("config ")[1].split(":")[0]), "packets": int(c["packets_per_gpu"]),
    "max_layers": int(c["max_layers"]), "checksums": bool(c["checksums"]), "layout": c.get("layout", "fixed"),
    "records": c.get("records", "summary"), "window": c.get("window", "default"), "sizes": c.get("sizes", "imix"),
    "kernel_sha": kernel_sha(),
    "fetch_size_kib": fetch_kib, "write_size_kib": write_kib, "launches": [nf, nw],
    "read_bytes_corrected": 2 * fetch_kib * 1024, "write_bytes": write_kib * 1024,
    "hbm_bytes_per_launch": int(2 * fetch_kib * 1024 + write_kib * 1024),
    "correction": "gfx950 FETCH_SIZE = half the bytes of 16B/lane streaming reads (MI355X_MICROARCH.md §HBM)",
}
Path(sys.argv[4]).write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out))
