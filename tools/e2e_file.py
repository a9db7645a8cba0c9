"""End-to-end rates from capture files (GPU box, repo root): packets start in a pcap file and end as parse records in
host memory (north_star: "the rate including the H2D/D2H copies must also be measured").

1. file -> records: BASELINE config 3's 10M-packet IMIX batch written as a pcap into /dev/shm (tmpfs), then
   examples/bin/pcap_parse -- the engine's reader (zero-copy map batches, or the copying reader into page-locked
   buffers with --copy) overlapped with pcppx_parse_batch_host (chunked H2D, parse on the GPU, D2H into page-locked
   record arrays) -- for 8 layer rows + checksums and for summaries only.
2. the reference's Google-benchmark parse loops (benchmark-google.cpp:15-64,149-264, examples/benchmark_google_loops.inc)
   over the facade (examples/bin/benchmark_google) beside the same loops over the reference Packet++
   (oracle/_ref/benchmark_google_ref), on example.pcap and the 10M IMIX pcap (--only google: this part alone).
3. the drop-in benchmark: examples/bin/benchmark (the reference's PcapPlusPlus-benchmark loop with the batch prepass)
   beside oracle/_ref/benchmark_ref (the reference's benchmark.cpp compiled unchanged, one core) on the config-1 10k
   pcap, the reference's example.pcap (frozen in tests/golden/capture_example.npz) and the 10M IMIX pcap.

  python tools/e2e_file.py --out gpurun_out/r03_e2e_file.json

E2E_ENGINE_GOOGLE / E2E_ENGINE_BENCH name another build of the engine's google-benchmark / drop-in program under
examples/bin (an A/B of facade variants on one box, e.g. the first-page size: profiles/r06u_fp_*, r06y_dropin_*).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from pcapplusplus_amd import synth  # noqa: E402
from pcapplusplus_amd.pcap import write_pcap  # noqa: E402


def run(cmd, timeout=600) -> str:
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise SystemExit(f"{cmd} failed ({r.returncode}): {r.stderr[-2000:]}")
    return r.stdout


def bench_pair(pcap: Path, reps: tuple[int, int], n: int, trials: int = 1) -> dict:
    """Per-run time of the reference benchmark and of the engine's drop-in, from two repetition counts (process
    start-up, file open and HIP initialisation cancel out), as tools/config1.py does. With trials > 1 the two programs
    alternate, trial by trial, and each reports the median of its trials (the box's host is shared: a lone pair of
    measurements can land in a busy second)."""
    out = {"packets": n, "pcap_bytes": pcap.stat().st_size}
    progs = [(name, exe) for name, exe in (("reference_benchmark", ROOT / "oracle" / "_ref" / "benchmark_ref"),
                                           ("engine_benchmark", ROOT / "examples" / "bin" /
                                            os.environ.get("E2E_ENGINE_BENCH", "benchmark")))
             if exe.exists()]
    per = {name: [] for name, _ in progs}
    inproc = {name: [] for name, _ in progs}
    last = {}
    for _ in range(trials):
        for name, exe in progs:
            walls = []
            for r in reps:
                t = time.perf_counter()
                last[name] = run([exe, pcap, "packet", r], timeout=1200).strip().splitlines()[-1]
                walls.append(time.perf_counter() - t)
            per[name].append((walls[1] - walls[0]) / (reps[1] - reps[0]) * 1e3)
            # the program's own figure (benchmark.cpp: whole ms of open-to-loop-end over the runs, / runs): exact enough
            # for runs of 100+ ms, where the process start-up noise left in the wall-clock difference is not
            inproc[name].append(float(last[name].split()[1]))
    for name, _ in progs:
        ms = sorted(per[name])[len(per[name]) // 2]
        ip = sorted(inproc[name])[len(inproc[name]) // 2]
        out[name] = {"ms_per_run": round(ms, 4), "Mpackets_per_s": round(n / ms / 1e3, 2), "stdout": last[name],
                     "threads": 1 if name == "reference_benchmark" else "1 host thread + mapper + parser threads + GPU",
                     "reps": list(reps), "trials_ms": [round(x, 4) for x in per[name]],
                     "in_process_ms_per_run": ip, "in_process_trials_ms": inproc[name],
                     "in_process_Mpackets_per_s": round(n / ip / 1e3, 2) if ip > 0 else None}
    if "reference_benchmark" in out and "engine_benchmark" in out:
        out["speedup"] = round(out["reference_benchmark"]["ms_per_run"] / out["engine_benchmark"]["ms_per_run"], 2)
        if out["engine_benchmark"]["in_process_ms_per_run"] > 0:
            out["in_process_speedup"] = round(out["reference_benchmark"]["in_process_ms_per_run"] /
                                              out["engine_benchmark"]["in_process_ms_per_run"], 2)
    return out


def google_pair(pcap: Path, args: list[str], trials: int = 1) -> dict:
    """The reference's Google-benchmark parse loops (examples/benchmark_google_loops.inc) over the engine's facade
    (examples/bin/benchmark_google) and over the reference Packet++ built from source (oracle/_ref/benchmark_google_ref,
    one core), alternating trial by trial; per benchmark the median of the trials' ns per iteration."""
    progs = [(name, exe) for name, exe in (("reference", ROOT / "oracle" / "_ref" / "benchmark_google_ref"),
                                           ("engine", ROOT / "examples" / "bin" / os.environ.get("E2E_ENGINE_GOOGLE",
                                                                                                  "benchmark_google")))
             if exe.exists()]
    per: dict = {}
    for _ in range(trials):
        for name, exe in progs:
            for ln in run([exe, "--pcap-file", pcap, *args], timeout=1500).strip().splitlines():
                d = json.loads(ln)
                if "name" in d and "ns_per_iteration" in d:
                    per.setdefault(d["name"].split("/")[0], {}).setdefault(name, []).append(d)
                elif "gpu_parses" in d:
                    per.setdefault("gpu_parses", []).append(d)
    out = {"file": pcap.name, "args": args, "trials": trials}
    for bm, by in per.items():
        if bm == "gpu_parses":
            out[bm] = by
            continue
        out[bm] = {}
        for name, ds in by.items():
            # BM_PacketFirstPass: one pass over the whole file per iteration, so per packet = per iteration / packets
            per_it = (ds[-1].get("items", ds[-1]["iterations"]) / ds[-1]["iterations"]) if bm == "BM_PacketFirstPass" else 1
            ns = sorted(round(d["ns_per_iteration"] / per_it, 3) for d in ds)
            out[bm][name] = {"ns_per_packet": ns[len(ns) // 2], "trials_ns": ns, "iterations": ds[-1]["iterations"]}
            if bm == "BM_PacketFirstPass":
                out[bm][name]["packets_per_pass"] = int(per_it)
        if "reference" in out[bm] and "engine" in out[bm]:
            out[bm]["speedup"] = round(out[bm]["reference"]["ns_per_packet"] / out[bm]["engine"]["ns_per_packet"], 2)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=10_000_000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--shm", default="/dev/shm")
    ap.add_argument("--only", choices=("all", "google", "dropin", "firstpass", "files"), default="all",
                    help="google: only the benchmark-google loops (example.pcap and the IMIX pcap); dropin: only the "
                         "drop-in benchmark.cpp runs (5 IMIX trials); firstpass: only the first-pass costs; files: only file -> records")
    args = ap.parse_args()
    res = {"cores": len(os.sched_getaffinity(0))}
    big = Path(args.shm) / f"pcppx_e2e_{os.getpid()}.pcap"
    exf = Path(args.shm) / f"pcppx_example_{os.getpid()}.pcap"
    try:
        t = time.time()
        b = synth.config(3, args.packets)
        write_pcap(big, b)
        res["imix_pcap"] = {"packets": b.n, "bytes": big.stat().st_size, "wire_bytes": int(b.caplens.sum()),
                            "gen_write_seconds": round(time.time() - t, 1), "where": "tmpfs (/dev/shm)"}
        del b
        print(json.dumps(res["imix_pcap"]), flush=True)
        from conftest import GOLDEN, load_golden

        ex, _ = load_golden(GOLDEN / "capture_example.npz")
        write_pcap(exf, ex)
        if args.only in ("all", "google", "firstpass"):
            # first-pass costs: BM_PacketFirstPass times the reader's open, the preload of every
            # packet (getNextPackets) and one Packet per packet -- the engine's GPU parse of the pages included -- each
            # repetition over a reader of its own; and the reference's BM_PacketPureParsing body run for exactly one pass
            # (--iterations = the file's packets), whose preload is untimed in both programs
            fp = {}
            for tag, f, n, reps in (("example_pcap", exf, ex.n, 7), ("imix_10M", big, args.packets, 3)):
                fp[tag] = google_pair(f, ["--benchmark", "BM_PacketFirstPass", "--iterations", "1", "--repetitions",
                                          str(reps)], trials=3 if tag == "example_pcap" else 1)
                fp[tag + "_pure_one_pass"] = google_pair(f, ["--benchmark", "BM_PacketPureParsing", "--iterations", str(n),
                                                             "--repetitions", str(reps)],
                                                         trials=3 if tag == "example_pcap" else 1)
                print("first_pass", tag, json.dumps(fp[tag]), flush=True)
            res["first_pass"] = fp
        if args.only in ("all", "google"):
            # benchmark-google.cpp's loops: all three on example.pcap (the library's 0.5-s runs); the two parse loops on
            # the IMIX pcap at fixed counts (the pure loop: three passes over the preloaded 10M packets)
            res["google_example_pcap"] = google_pair(exf, ["--min-time", "0.5"], trials=3)
            print("google_example", json.dumps(res["google_example_pcap"]), flush=True)
            res["google_imix_pure"] = google_pair(big, ["--benchmark", "BM_PacketPureParsing", "--iterations",
                                                        str(3 * args.packets)])
            print("google_imix_pure", json.dumps(res["google_imix_pure"]), flush=True)
            res["google_imix_parsing"] = google_pair(big, ["--benchmark", "BM_PacketParsing", "--iterations",
                                                           str(args.packets)])
            print("google_imix_parsing", json.dumps(res["google_imix_parsing"]), flush=True)
        if args.only in ("all", "files"):
            runs = {}
            for tag, extra in (("map_l8_csum", []), ("copy_l8_csum", ["--copy"]),
                               ("map_summary", ["--layers", "0", "--checksums", "0"]),
                               ("copy_summary", ["--copy", "--layers", "0", "--checksums", "0"])):
                line = run([ROOT / "examples" / "bin" / "pcap_parse", big, "--reps", "3", *extra], timeout=900)
                runs[tag] = json.loads(line.strip().splitlines()[-1])
                print(tag, json.dumps(runs[tag]), flush=True)
            res["file_to_records"] = runs
        if args.only in ("all", "dropin"):
            # the drop-in benchmark beside the reference's own (and the round-4 drop-in where built), same host
            c1 = Path(args.shm) / f"pcppx_cfg1_{os.getpid()}.pcap"
            b1 = synth.config(1)
            write_pcap(c1, b1)
            try:
                # 2,000 runs apart: the start-up noise of a process (HIP initialisation, +-0.1 s) is 0.05 ms per run
                res["benchmark_config1"] = bench_pair(c1, (10, 2010), b1.n, trials=7)
            finally:
                c1.unlink()
            print("config1", json.dumps(res["benchmark_config1"]), flush=True)
            res["benchmark_example_pcap"] = bench_pair(exf, (10, 2010), ex.n, trials=7)
            print("example.pcap", json.dumps(res["benchmark_example_pcap"]), flush=True)
            res["benchmark_imix_10M"] = bench_pair(big, (1, 5), args.packets, trials=5 if args.only == "dropin" else 3)
            print("imix", json.dumps(res["benchmark_imix_10M"]), flush=True)
    finally:
        big.unlink(missing_ok=True)
        exf.unlink(missing_ok=True)
    line = json.dumps(res, indent=1)
    if args.out:
        Path(args.out).write_text(line + "\n")
    print(line)


if __name__ == "__main__":
    main()
