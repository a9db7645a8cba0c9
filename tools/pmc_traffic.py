"""HBM traffic per launch of the parse kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py.

gfx950 correction (/opt/skills/guides/MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half of the
bytes of a wide (16 B/lane) coalesced streaming read; WRITE_SIZE is exact for 16-B-per-lane stores. Both
are in KiB. Our reads are dwordx4 (16 B/lane) loads, so hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024.
The result is keyed by everything bench.py checks before using it: config, packets, max_layers, checksums and the
sha of the kernel source it was measured on (bench.kernel_sha).

  python tools/pmc_traffic.py <fetch_dir> <write_dir> <config> <packets> <max_layers> <checksums 0|1> <out.json>
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
out = {
    "config": int(sys.argv[3]), "packets": int(sys.argv[4]), "max_layers": int(sys.argv[5]),
    "checksums": sys.argv[6] == "1", "kernel_sha": kernel_sha(),
    "fetch_size_kib": fetch_kib, "write_size_kib": write_kib, "launches": [nf, nw],
    "read_bytes_corrected": 2 * fetch_kib * 1024, "write_bytes": write_kib * 1024,
    "hbm_bytes_per_launch": int(2 * fetch_kib * 1024 + write_kib * 1024),
    "correction": "gfx950 FETCH_SIZE = half the bytes of 16B/lane streaming reads (MI355X_MICROARCH.md §HBM)",
}
Path(sys.argv[7]).write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out))
