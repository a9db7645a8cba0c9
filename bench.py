"""bench.py — device-resident Packet++ parse throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]): a 10M-packet IMIX batch (64/512/1500 B at
7:4:1; 25% VLAN; 70% IPv4 / 30% IPv6; TCP/UDP 50/50; 1% corrupted checksums), synthetic, seed 3 (+rank).
One step = one pass of the parse kernel over the whole batch already resident in HBM: layer chain
(8 layer records/packet), hash5Tuple both directions, hash2Tuple, IPv4 + TCP/UDP checksum verify.

Multi-GPU: one process per GPU (torch.distributed, launched by torch.distributed.run); packets are
independent, so each rank parses its own 10M-packet shard with no data-path collective ("weak").
Rank 0 prints one JSON line. value = packets of all ranks / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md (Chip-level parameters)
DESC_BYTES = 12          # u64 offset + u32 caplen per packet


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--packets", type=int, default=10_000_000, help="packets per GPU")
    ap.add_argument("--config", type=int, default=3, choices=(2, 3, 4))
    ap.add_argument("--max-layers", type=int, default=8)
    ap.add_argument("--no-checksums", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="packets in the CPU-baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="min CPU-baseline time (repeat passes)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="also time the host-to-host (PCIe-inclusive) path")
    ap.add_argument("--traffic", default=str(ROOT / "profiles" / "r01_traffic.json"),
                    help="PMC-derived HBM bytes per launch (from tools/pmc_traffic.py)")
    return ap.parse_args()


def algorithmic_read_bytes(batch, want_checksums: bool, summary) -> int:
    """checksum runs read every caplen byte; otherwise bytes up to the end of the last
    parsed L2-L4 header; plus a 12-B descriptor per packet."""
    if want_checksums:
        return int(batch.caplens.sum(dtype=np.int64)) + DESC_BYTES * batch.n
    raise NotImplementedError("no-checksum byte model needs the header extent")


def cpu_baseline(batch, opts, sample: int, min_seconds: float) -> dict:
    import oracle  # test infrastructure: the checker, timed here only as the reported CPU baseline

    sub = batch.slice(0, min(sample, batch.n))
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, 16))
    kind = "reference" if oracle.ref_available() else "port"
    fn = oracle.ref_bench if kind == "reference" else oracle.oracle_bench
    total_t, total_p = 0.0, 0
    while total_t < min_seconds:
        t, _ = fn(sub, opts, threads)
        total_t += t
        total_p += sub.n
    return {"value": round(total_p / total_t / 1e6, 3), "unit": "Mpackets/s", "cores": threads, "kind": kind,
            "sample": f"first {sub.n} packets of the same batch, {total_p // sub.n} passes, "
                      f"{total_t:.1f} s; {'reference Packet++ built from source' if kind == 'reference' else 'C restatement'}"
                      f": Packet(&raw) + hash5Tuple x2 + hash2Tuple + IPv4/L4 checksums, {threads} threads"}


def main() -> None:
    args = parse_args()
    import torch
    import torch.distributed as dist

    from pcapplusplus_amd import abi, shard, synth
    from pcapplusplus_amd.engine import Engine, to_device

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = f"cuda:{local}"
    torch.cuda.set_device(dev)

    # ---- synthetic shard for this rank (per-GPU work fixed: weak scaling) ----
    t0 = time.time()
    if args.config == 3:
        batch = synth.imix(args.packets, shard.shard_seed(3, rank))
    elif args.config == 4:
        batch = synth.imix(args.packets, shard.shard_seed(4, rank), flows=1_000_000, corrupt_frac=0.0)
    else:
        batch = synth.small64(args.packets, shard.shard_seed(2, rank))
    gen_s = time.time() - t0
    want_csum = not args.no_checksums
    opts = abi.make_opts(0, 8, want_csum, args.max_layers)
    n = batch.n
    eng = Engine(local)
    data, offsets, caplens = to_device(batch, dev)
    summary = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    layers = torch.empty(max(n * args.max_layers, 1) * 8, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step():
        eng.parse_device(data, offsets, caplens, n, batch.linktype, opts, summary, layers, sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    w0 = time.perf_counter()
    for k in range(args.steps):
        starts[k].record(stream)
        step()
        ends[k].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - w0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))

    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max, kern_max = float(t[0]), float(t[1])
    total_packets = n * world * args.steps
    mpps = total_packets / wall_max / 1e6
    wire = int(batch.caplens.sum(dtype=np.int64))
    read_bytes = algorithmic_read_bytes(batch, want_csum, None)
    write_bytes = n * (32 + 8 * args.max_layers)
    achieved = read_bytes / (kern_ms * 1e-3) / 1e9

    # sanity: the records of the last step parse every packet cleanly (synthetic data has no L7 triggers)
    s = summary.view(torch.int32).view(n, 8)
    flags = (s[:, 3] & 0xFFFF)
    flagged = int(((flags & abi.F_NEEDS_HOST) != 0).sum().item())

    traffic = None
    tp = Path(args.traffic)
    if tp.exists():
        try:
            tj = json.loads(tp.read_text())
            if tj.get("packets") == n and tj.get("config") == args.config and tj.get("max_layers") == args.max_layers:
                traffic = tj.get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    e2e = None
    if args.e2e and rank == 0:
        sub = batch.slice(0, min(n, 2_000_000))
        eng.parse_host(sub, opts)
        t1 = time.perf_counter()
        eng.parse_host(sub, opts)
        e2e_t = time.perf_counter() - t1
        e2e = {"Mpackets_per_s": round(sub.n / e2e_t / 1e6, 2),
               "wire_GBps": round(int(sub.caplens.sum(dtype=np.int64)) / e2e_t / 1e9, 2), "packets": sub.n}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(batch, opts, args.cpu_sample, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "Mpackets/s + GB/s device-resident parse, 64B-1500B IMIX, 1/2/4/8 MI355X",
            "value": round(mpps, 2),
            "unit": "Mpackets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": f"config {args.config}: {n} packets/GPU " + (
                    "IMIX 64/512/1500 B 7:4:1, 25% VLAN, 70/30 IPv4/IPv6, TCP/UDP 50/50, 1% bad checksums"
                    if args.config == 3 else "see synth.py"),
                "packets_per_gpu": n,
                "wire_bytes_per_gpu": wire,
                "checksums": want_csum,
                "max_layers": args.max_layers,
                "parallelism": f"shard{world} (no collective)",
                "wire_GBps": round(wire * world * args.steps / wall_max / 1e9, 2),
                "kernel_ms": round(kern_max, 4),
                "flagged_packets": flagged,
                "gen_seconds": round(gen_s, 1),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "algorithmic_read_bytes": read_bytes,
                "record_write_bytes": write_bytes,
            },
            "cpu_baseline": cpu,
        }
        if e2e is not None:
            line["e2e_host_to_host"] = e2e
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
