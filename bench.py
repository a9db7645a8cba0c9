"""bench.py — device-resident Packet++ parse throughput on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[2]): a 10M-packet IMIX batch (64/512/1500 B
at 7:4:1; 25% VLAN; 70% IPv4 / 30% IPv6; TCP/UDP 50/50; 1% corrupted checksums), synthetic, seed 3 (+rank).
One step = one pass of the parse kernel over the whole batch already resident in HBM: layer chain
(up to 8 layer records/packet, PACKED), hash5Tuple both directions, hash2Tuple, IPv4 + TCP/UDP checksum verify; records:
the 16-B brief per packet (hashes, flags incl. the checksum verdicts, chain length, port layer) + the layer rows.

--config selects the other BASELINE configs as extra bench lines (not the driver's default):
  2: 1M x 64 B Eth/IPv4/{TCP,UDP}: parse + hash5Tuple (5-tuple extract), no checksums;
  4: 12.5M IMIX packets/GPU with Zipf(1.1) 5-tuples over 1M flows: parse + hash5Tuple + per-flow
     {packets, bytes} counters in an HBM flow table (DpdkExample-FilterTraffic's flow table); the ranks' shards are
     contiguous ranges of ONE stream over ONE flow universe (synth.flow_stream), merged on the host after timing;
  5: 10M deep-encapsulation packets (QinQ / MPLS stacks / GREv0 / IPv6 extension chains): parse + hashes.
Without checksums the algorithmic read is each packet's header extent (end of its last L2-L4 header,
SURVEY.md §8d) + the 12-B descriptor, computed from the records the kernel wrote.

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
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--packets", type=int, default=None, help="packets per GPU (default: the config's size)")
    ap.add_argument("--config", type=int, default=3, choices=(2, 3, 4, 5))
    ap.add_argument("--sizes", choices=("imix", "64", "512", "1500"), default="imix",
                    help="config 3's packet sizes: the 64/512/1500-B IMIX at 7:4:1 (the headline), or one size only (the "
                         "north star's per-size batches: same VLAN / IPv4 / IPv6 / TCP / UDP mix and checksum verify; "
                         f"packets per GPU {SIZED_PACKETS})")
    ap.add_argument("--max-layers", type=int, default=None,
                    help="layer records per packet (default: 8 for config 3, 12 for config 5, 0 for the configs whose "
                         "consumer reads no layers: 2's 5-tuple extract, 4's flow table)")
    ap.add_argument("--checksums", choices=("auto", "on", "off"), default="auto",
                    help="IPv4/L4 checksum verify (auto: on for config 3 only)")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="packets in the CPU-baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="min CPU-baseline time (repeat passes)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-to-host (PCIe-inclusive) timing")
    ap.add_argument("--traffic", default=None,
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py; default profiles/traffic_cfg<N>.json); "
                         "used only if it was measured on this kernel source, config, size and record options")
    ap.add_argument("--no-traffic", action="store_true", help="do not report PMC traffic (the PMC passes themselves)")
    ap.add_argument("--window", choices=("auto", "default", "deep", "short"), default="auto",
                    help="the header window the parse gathers (pcppx_opts.window; records identical): deep = two-round "
                         "144 B for checksum launches over deep stacks, short = one 96-B round for parse-only launches over "
                         "plain stacks (auto: " + ", ".join(f"config {c} {v}" for c, v in sorted(CONFIG_WINDOW.items())) +
                         ", else default)")
    ap.add_argument("--layout", choices=("auto", "fixed", "packed"), default="auto",
                    help="layer-record layout (pcppx_opts.layout): fixed = max_layers entries per packet; packed = only the "
                         "chain's entries, dense per 64-packet tile (the same entries; auto: " + ", ".join(
                             f"config {c} {v}" for c, v in sorted(CONFIG_LAYOUT.items())) + ")")
    ap.add_argument("--records", choices=("auto", "summary", "brief", "tuples", "keys"), default="auto",
                    help="per-packet record: the 32-B summary, the 16-B brief (pcppx_brief: the summary's first half -- "
                         "hashes, flags incl. the checksum verdicts, chain length, port layer; isPacketOfType from the "
                         "layer rows), the 48-B 5-tuple extract (pcppx_tuple) alone, or (config 4) only what the flow table "
                         "reads: the dense hash5 column + collectStats, no summary (auto: " + ", ".join(
                             f"config {c} {v}" for c, v in sorted(CONFIG_RECORDS.items())) + ")")
    ap.add_argument("--dump-flows", default=None,
                    help="config 4: write the merged flow table (rank 0, after the timed region) to this .npz")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="gloo: a multi-rank rehearsal on fewer GPUs than ranks (ranks share cards round-robin); "
                         "the timed numbers of such a run are not a scaling measurement")
    return ap.parse_args()


CONFIG_PACKETS = {2: 1_000_000, 3: 10_000_000, 4: 12_500_000, 5: 10_000_000}
SIZED_PACKETS = {64: 10_000_000, 512: 10_000_000, 1500: 5_000_000}  # config 3 at one size: 0.6 / 5.1 / 7.5 GB per GPU
CONFIG_MAX_LAYERS = {2: 0, 3: 8, 4: 0, 5: 12}
CONFIG4_FLOWS = 1_000_000  # config 4's flow universe (one for all ranks)
CONFIG_LAYOUT = {3: "packed", 5: "packed"}  # configs with layer records
# per-packet records: config 2 the 5-tuple extract its name asks for; configs 3 / 5 the 16-B brief beside the layer rows
# (hashes, flags with the checksum verdicts, chain length, port layer; isPacketOfType from the rows -- ABI 7); config 4
# what the flow table reads
CONFIG_RECORDS = {2: "tuples", 3: "brief", 4: "keys", 5: "brief"}
# plain Eth / VLAN / IP / L4 stacks (configs 2 and 4): the one-round parse-only window (PCPPX_WINDOW_SHORT)
CONFIG_WINDOW = {2: "short", 4: "short"}
KERNEL_SRC = ROOT / "pcapplusplus_amd" / "csrc" / "pcppx_kernels.hip"


def kernel_sha() -> str:
    """Identity of the kernel source a traffic measurement belongs to."""
    import hashlib

    return hashlib.sha256(KERNEL_SRC.read_bytes()).hexdigest()[:16]


def load_traffic(path: Path, cfg: int, n: int, ml: int, csum: bool, layout: str = "fixed",
                 records: str = "summary", window: str = "default", sizes: str = "imix") -> tuple[int | None, str]:
    """(HBM bytes per parse launch, note) from a PMC traffic file, only if it matches this run exactly."""
    if not path.exists():
        return None, f"no PMC measurement ({path.name})"
    try:
        tj = json.loads(path.read_text())
    except (ValueError, OSError) as e:
        return None, f"unreadable {path.name}: {e}"
    want = {"config": cfg, "packets": n, "max_layers": ml, "checksums": csum, "layout": layout, "records": records,
            "window": window, "sizes": sizes,
            "kernel_sha": kernel_sha()}
    got = {k: tj.get(k, {"layout": "fixed", "records": "summary", "window": "default", "sizes": "imix"}.get(k))
           for k in want}
    if got != want:
        return None, f"stale {path.name}: measured {got}, this run {want}"
    return int(tj["hbm_bytes_per_launch"]), f"{path.name} (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE)"


def cpu_cores() -> tuple[int, str]:
    """Host cores this process may use: the affinity mask, capped by a cgroup CPU quota (a GPU box's share)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    if quota is not None and quota < aff:
        return quota, f"{quota} of {aff} affinity cores (cgroup cpu.max quota)"
    return aff, f"all {aff} cores of the affinity mask"
WORKLOADS = {
    2: "config 2: 64 B Eth/IPv4/{TCP,UDP} 50/50; parse + hash5Tuple, 5-tuple extract",
    3: "config 3: IMIX 64/512/1500 B 7:4:1, 25% VLAN, 70/30 IPv4/IPv6, TCP/UDP 50/50, 1% bad checksums; "
       "parse + hashes + IPv4/L4 checksum verify",
    4: "config 4: IMIX as config 3 with 5-tuples Zipf(1.1) over 1M flows, both directions, one stream cut into "
       "contiguous per-GPU shards; parse + hash5Tuple + "
       "per-flow {packets, bytes} counters (FilterTraffic flow table) + collectStats protocol histogram",
    5: "config 5: deep encapsulation (QinQ, 1-3 MPLS labels, GREv0 C/K/S over IPv4|IPv6, IPv6 1-3 extension "
       "headers) then TCP/UDP, 64/512/1500 B; parse + hashes",
}


def algorithmic_read_bytes(batch, want_checksums: bool, summary=None, layers=None, caplens=None,
                           max_layers: int = 0) -> int:
    """checksum runs read every caplen byte; otherwise the bytes up to the end of the last
    parsed L2-L4 header (from the layer records: max over non-Payload, non-Trailer layers of offset +
    hdr_len, capped at caplen); plus a 12-B descriptor per packet."""
    if want_checksums:
        return int(batch.caplens.sum(dtype=np.int64)) + DESC_BYTES * batch.n
    import torch

    n, ml = batch.n, max_layers
    lay = layers[: n * ml * 8].view(n, ml, 8).to(torch.int32)
    proto = lay[:, :, 0]
    end = (lay[:, :, 2] | (lay[:, :, 3] << 8)) + (lay[:, :, 4] | (lay[:, :, 5] << 8))
    nl = summary.view(n, 32)[:, 14].to(torch.int32)
    k = torch.arange(ml, device=layers.device, dtype=torch.int32)
    valid = (k[None, :] < nl[:, None]) & (proto != 25) & (proto != 30)
    ext = torch.where(valid, end, torch.zeros_like(end)).amax(dim=1)
    ext = torch.minimum(ext, caplens.to(torch.int32))
    return int(ext.sum(dtype=torch.int64).item()) + DESC_BYTES * n


def cpu_baseline(batch, opts, sample: int, min_seconds: float) -> dict:
    import oracle  # test infrastructure: the checker, timed here only as the reported CPU baseline

    sub = batch.slice(0, min(sample, batch.n))
    threads, core_note = cpu_cores()
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
                      f": Packet(&raw) + hash5Tuple x2 + hash2Tuple"
                      f"{' + IPv4/L4 checksums' if opts.want_checksums else ''}, {threads} threads = {core_note}"}


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(gpus: int, argv: list[str], port: int) -> list[str]:
    """The child command that runs `bench.py <argv>` as `gpus` ranks, one process per GPU on this node
    (the reference's one-worker-per-core launch, Pcap++/src/DpdkDeviceList.cpp:346-440)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]


def check_world(gpus: int, env) -> int | None:
    """None when this process is a rank of a `gpus`-rank job (or a 1-GPU run); otherwise an exit code.
    A rank whose WORLD_SIZE differs from --gpus would report a GPU count nobody asked for."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return None if gpus == 1 else 0  # 0: not a rank yet; the caller launches the ranks
    if int(ws) != gpus:
        print(f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}: refusing to report a {ws}-rank run as {gpus} GPUs",
              file=sys.stderr, flush=True)
        return 2
    return None


def launch_ranks(gpus: int, argv: list[str]) -> int:
    """Parent of an N-GPU run: starts the N ranks as a child torch.distributed.run and forwards their output
    and exit code. This process never imports torch or touches the GPU (no exec after GPU initialisation)."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = launcher_cmd(gpus, argv, free_port())
    print("bench.py: launching " + " ".join(cmd[1:]), file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    assert proc.stdout is not None
    for line in proc.stdout:  # rank 0's JSON line (and anything else the ranks print), as it arrives
        sys.stdout.write(line)
        sys.stdout.flush()
    return proc.wait()


def main() -> None:
    args = parse_args()
    rc = check_world(args.gpus, os.environ)
    if rc is not None:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]) if rc == 0 else rc)
    import torch
    import torch.distributed as dist

    from pcapplusplus_amd import abi, shard, synth
    from pcapplusplus_amd.engine import Engine, to_device

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.dist_backend == "gloo":
        local = local % torch.cuda.device_count()  # rehearsal: ranks share the card(s)
    elif world > 1 and world > torch.cuda.device_count():
        print(f"bench.py: {world} ranks over RCCL need {world} GPUs, this node has {torch.cuda.device_count()} "
              f"(--dist-backend gloo rehearses more ranks than GPUs)", file=sys.stderr, flush=True)
        sys.exit(2)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")
    dev = f"cuda:{local}"
    torch.cuda.set_device(dev)

    # ---- synthetic shard for this rank (per-GPU work fixed: weak scaling) ----
    cfg = args.config
    if args.sizes != "imix" and cfg != 3:
        sys.exit("bench.py: --sizes selects config 3's packet size")
    sized = int(args.sizes) if args.sizes != "imix" else None
    npk = args.packets or (SIZED_PACKETS[sized] if sized else CONFIG_PACKETS[cfg])
    ml = args.max_layers if args.max_layers is not None else CONFIG_MAX_LAYERS[cfg]
    t0 = time.time()
    seed = shard.shard_seed(cfg, rank)
    if cfg == 3:
        batch = synth.imix(npk, seed, sizes=(sized,), weights=(1,)) if sized else synth.imix(npk, seed)
    elif cfg == 4:
        # one config-4 stream over one 1M-flow universe, cut into contiguous shards: rank r parses packets
        # [npk*r, npk*(r+1)) of it, so a flow spans ranks and the host merge adds them up
        batch = synth.flow_stream(npk * rank, npk * (rank + 1), 4, flows=CONFIG4_FLOWS)
    elif cfg == 5:
        batch = synth.deep(npk, seed)
    else:
        batch = synth.small64(npk, seed)
    gen_s = time.time() - t0
    want_csum = args.checksums == "on" or (args.checksums == "auto" and cfg == 3)
    layout = args.layout if args.layout != "auto" else CONFIG_LAYOUT.get(cfg, "fixed")
    rec_kind = args.records if args.records != "auto" else CONFIG_RECORDS[cfg]
    if rec_kind == "brief" and not ml:
        sys.exit("bench.py: --records brief goes with layer records (isPacketOfType comes from them)")
    if rec_kind in ("tuples", "keys") and ml:
        sys.exit(f"bench.py: --records {rec_kind} writes no layer records (use --max-layers 0)")
    if rec_kind == "keys" and cfg != 4:
        sys.exit("bench.py: --records keys is config 4's flow-table launch")
    window = args.window if args.window != "auto" else CONFIG_WINDOW.get(cfg, "default")
    opts = abi.make_opts(0, 8, want_csum, ml, {"default": abi.WINDOW_DEFAULT, "deep": abi.WINDOW_DEEP,
                                               "short": abi.WINDOW_SHORT}[window],
                         {"fixed": abi.LAYOUT_FIXED, "packed": abi.LAYOUT_PACKED}[layout])
    n = batch.n
    eng = Engine(local)
    data, offsets, caplens = to_device(batch, dev)
    summary = torch.empty(n * 32, dtype=torch.uint8, device=dev) if rec_kind == "summary" else None
    brief = torch.empty(n * 16, dtype=torch.uint8, device=dev) if rec_kind == "brief" else None
    tuples = torch.empty(n * 48, dtype=torch.uint8, device=dev) if rec_kind == "tuples" else None
    layers = torch.empty(max(n * ml, 1) * 8, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    flows = None
    flow_keys = None
    proto_stats = None
    if cfg == 4:  # per-GPU flow table: 2M slots for 1M flows, counters accumulate over all steps
        cap = 1 << 21
        flows = (torch.zeros(cap, dtype=torch.int32, device=dev), torch.zeros(cap, dtype=torch.int64, device=dev),
                 torch.zeros(cap, dtype=torch.int64, device=dev), torch.zeros(4, dtype=torch.int64, device=dev), cap)
        # the parse also writes the dense hash5 column the flow table is keyed by (pcppx_records.flow_keys) and the
        # collectStats protocol counters (pcppx_records.proto_stats, accumulated over every launch)
        flow_keys = torch.empty(n, dtype=torch.int32, device=dev)
        proto_stats = torch.zeros(abi.PROTO_STATS, dtype=torch.int64, device=dev)
    mids = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)] if flows else None

    def step(k=None):
        eng.parse_device(data, offsets, caplens, n, batch.linktype, opts, summary, layers, sh, flow_keys, tuples,
                         proto_stats, brief)
        if flows is not None:
            if k is not None:
                mids[k].record(stream)
            keys, pk, by, st, cap = flows
            eng.flow_count_keys_device(flow_keys, caplens, n, keys, pk, by, cap, st, sh)

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
        step(k)
        ends[k].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - w0
    step_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))
    # the parse kernel is the dominant kernel of every config; config 4 also runs the flow-table kernels
    kern_each = [s.elapsed_time(e) for s, e in zip(starts, mids if mids else ends)]
    kern_ms = float(np.mean(kern_each))
    flow_ms = step_ms - kern_ms if mids else None

    tdev = dev if args.dist_backend == "nccl" else "cpu"
    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=tdev)
    per_rank = [t.clone() for _ in range(world)]
    if world > 1:
        dist.all_gather(per_rank, t)  # after the timed region: each rank's wall and kernel time
    per_rank = [[float(v) for v in x.cpu()] for x in per_rank]
    wall_max = max(p[0] for p in per_rank)
    kern_max = max(p[1] for p in per_rank)
    total_packets = n * world * args.steps
    mpps = total_packets / wall_max / 1e6
    wire = int(batch.caplens.sum(dtype=np.int64))
    # the records' chain lengths (packed write bytes), the flag check and -- for parse-only runs -- the header extents
    # (their byte model): from the timed run's own summary when it has one and computes checksums; else from one
    # untimed parse with full FIXED records through the checksum instance (the same records; for a checksum run that
    # writes no summary -- configs 3 with the brief -- the same kernel, launched once after the timed region:
    # tools/timed_stats.py keeps launches warmup+1 .. warmup+steps)
    if want_csum and summary is not None:
        ext_sum = summary
        read_bytes = algorithmic_read_bytes(batch, True)
    else:
        ext_sum = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        ext_lay = torch.empty(n * 16 * 8, dtype=torch.uint8, device=dev)
        eng.parse_device(data, offsets, caplens, n, batch.linktype, abi.make_opts(0, 8, True, 16), ext_sum, ext_lay, sh)
        torch.cuda.synchronize(dev)
        read_bytes = algorithmic_read_bytes(batch, want_csum, ext_sum, ext_lay, caplens, 16)
        del ext_lay
    nl16 = ext_sum.view(n, 32)[:, 14].to(torch.int64)
    chain_entries = int(torch.clamp(nl16, max=ml).sum().item()) if ml else 0
    per_pkt = (32 if summary is not None else 0) + (16 if brief is not None else 0) + \
        (48 if tuples is not None else 0) + (4 if flow_keys is not None else 0)
    write_bytes = n * per_pkt + {"fixed": 8 * n * ml, "packed": 8 * chain_entries}[layout]
    achieved = read_bytes / (kern_ms * 1e-3) / 1e9

    # sanity: every packet parses cleanly (synthetic data has no L7 triggers)
    s = ext_sum.view(torch.int32).view(n, 8)
    flags = (s[:, 3] & 0xFFFF)
    flagged = int(((flags & abi.F_NEEDS_HOST) != 0).sum().item())
    if tuples is not None:  # the timed output itself: every packet carries its 5-tuple, hash5 as the summary's
        tv = tuples.view(torch.int32).view(n, 12)
        tuple_check = {"with_5tuple": int(((tv[:, 9] >> 24) & 0xFF).eq(1).sum().item()),
                       "hash5_equal_summary": bool(torch.equal(tv[:, 10], s[:, 0]))}
    else:
        tuple_check = None
    # the flow table's keys: the timed launches' dense hash5 column equals the full parse's summary hash5
    keys_equal = bool(torch.equal(flow_keys, s[:, 0])) if flow_keys is not None else None
    # the timed launches' briefs: the first half of the full parse's summaries, byte for byte (a parse-only run against
    # the checksum parse above: but for its checksum flags)
    brief_equal = None
    if brief is not None:
        want16 = ext_sum.view(n, 32)[:, :16].clone()
        if not want_csum:
            csum_flags = abi.F_IP_CSUM | abi.F_IP_CSUM_OK | abi.F_L4_CSUM | abi.F_L4_CSUM_OK
            w = want16.view(torch.int32)
            w[:, 3] &= ~csum_flags
        brief_equal = bool(torch.equal(brief.view(n, 16), want16))
    stats_line = None
    if proto_stats is not None:  # collectStats over every launch (warmup + timed): the histogram of one pass
        launches = args.warmup + args.steps
        tot = proto_stats.cpu().numpy()
        consistent = bool((tot % launches == 0).all() and int(tot[0]) // launches == n)
        if world > 1:
            # every rank's PacketStats summed, as FilterTraffic sums its per-core stats at exit
            # (Examples/DpdkExample-FilterTraffic/main.cpp:279-287); after the timed region
            tt = torch.tensor(np.concatenate([tot, [1 if consistent else 0]]).astype(np.int64), device=tdev)
            dist.all_reduce(tt, op=dist.ReduceOp.SUM)
            tot, consistent = tt[:-1].cpu().numpy(), int(tt[-1]) == world
        stats_line = {f: int(tot[k]) // launches for k, f in enumerate(abi.PROTO_STATS_FIELDS)}
        stats_line["launches_per_rank"] = launches
        stats_line["ranks_merged"] = world
        stats_line["consistent"] = consistent and stats_line["packet_count"] == n * world
    del ext_sum

    traffic, traffic_note = None, "not requested"
    if not args.no_traffic:
        tag = f"{cfg}s{sized}" if sized else f"{cfg}"
        tp = Path(args.traffic) if args.traffic else ROOT / "profiles" / f"traffic_cfg{tag}.json"
        traffic, traffic_note = load_traffic(tp, cfg, n, ml, want_csum, layout, rec_kind, window, args.sizes)

    e2e = None
    if not args.no_e2e and rank == 0 and world == 1:
        # packets start and end in host memory: pcppx_parse_batch_host on the first 2M packets. pageable: input and
        # records in ordinary memory (staged / drained by host threads); pinned: input in page-locked memory (a NIC
        # ring: DMA from the caller's bytes); pinned_io: records returned into page-locked arrays too. Output arrays
        # are allocated once, outside the timed passes. Never `value`.
        from pcapplusplus_amd.engine import pinned_copy, pinned_records

        sub = batch.slice(0, min(n, 2_000_000))
        e2e = {"packets": sub.n, "max_layers": ml, "checksums": want_csum, "layout": "fixed"}
        # the host path returns the fixed layout and the summary (its records are the device path's, bit for bit)
        hopts = abi.make_opts(0, 8, want_csum, ml, opts.window)
        wire_sub = int(sub.caplens.sum(dtype=np.int64))
        for kind in ("pageable", "pinned", "pinned_io"):
            b2, buf = (sub, None) if kind == "pageable" else pinned_copy(sub)
            if kind == "pinned_io":
                out, keep = pinned_records(sub.n, ml)
            else:
                out, keep = (np.zeros(sub.n, dtype=abi.SUMMARY_DTYPE),
                             np.zeros(max(1, sub.n * ml), dtype=abi.LAYER_DTYPE)), None
            eng.parse_host(b2, hopts, out)
            reps = []
            for _ in range(3):  # median of 3 host-to-host passes (host threads make single passes noisy)
                t1 = time.perf_counter()
                eng.parse_host(b2, hopts, out)
                reps.append(time.perf_counter() - t1)
            e2e_t = float(np.median(reps))
            e2e[kind] = {"Mpackets_per_s": round(sub.n / e2e_t / 1e6, 2), "wire_GBps": round(wire_sub / e2e_t / 1e9, 2)}
            if buf is not None:
                buf.free()
            for k in keep or ():
                k.free()

    flow_check = None
    if flows is not None:
        # FilterTraffic's exit step (Examples/DpdkExample-FilterTraffic/main.cpp:279-287): every GPU's flow table is
        # merged by key on the host (after the timed region; nothing crosses GPUs on the data path). Conservation:
        # every packet of every launch on every rank is in a flow, the key-0 bucket or the no-free-slot count.
        keys, pk, by, st, cap = flows
        mine = shard.compact_device_table(keys.cpu().numpy(), pk.cpu().numpy(), by.cpu().numpy(), st.cpu().numpy())
        tables = [mine]
        if world > 1:
            tables = [None] * world
            dist.all_gather_object(tables, mine)
        if rank == 0:
            merged = shard.merge_device_tables(tables)
            counted = int(merged["packets"].sum()) + merged["key0_packets"] + merged["dropped"]
            expected = n * world * (args.warmup + args.steps)
            if args.dump_flows:
                np.savez(args.dump_flows, keys=merged["keys"], packets=merged["packets"], bytes=merged["bytes"],
                         key0=np.array([merged["key0_packets"], merged["key0_bytes"], merged["dropped"]], np.uint64),
                         launches=np.array([args.warmup + args.steps]))
            flow_check = {"merged_flows": int(len(merged["keys"])), "ranks_merged": len(tables),
                          "stream": f"one seed-4 stream over {CONFIG4_FLOWS} flows; rank r = packets [{n}r, {n}(r+1))",
                          "flow_universe": CONFIG4_FLOWS,
                          "merged_within_universe": int(len(merged["keys"])) <= CONFIG4_FLOWS,
                          "flows_spanning_ranks": int(sum(len(t["keys"]) for t in tables) - len(merged["keys"])),
                          "per_rank_flows": [int(len(t["keys"])) for t in tables],
                          "packets_counted": counted, "expected": expected, "conserved": counted == expected,
                          # exact: no packet fell to the no-free-slot count, i.e. the table is the reference's map
                          "exact": merged["dropped"] == 0,
                          "table_full_drops": merged["dropped"], "flow_kernel_ms": round(flow_ms, 4)}
            if merged["dropped"]:
                print(f"bench.py: flow table lost {merged['dropped']} packets (no free slot): per-flow counters are "
                      f"not the reference's", file=sys.stderr, flush=True)

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region (every rank's), so N>1 lines carry it too
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
                "workload": f"{n} packets/GPU, " + (WORKLOADS[cfg] if not sized else WORKLOADS[cfg].replace(
                    "IMIX 64/512/1500 B 7:4:1", f"{sized} B packets only (IMIX mix of stacks)")),
                "sizes": args.sizes,
                "packets_per_gpu": n,
                "wire_bytes_per_gpu": wire,
                "checksums": want_csum,
                "window": window,
                "max_layers": ml,
                "layout": layout,
                "records": rec_kind,
                "parallelism": f"shard{world} (no collective)",
                "ranks": world,
                "dist_backend": args.dist_backend if world > 1 else None,
                "per_rank_kernel_ms": [round(p[1], 4) for p in per_rank],
                "per_rank_wall_ms_per_step": [round(p[0] * 1e3 / args.steps, 4) for p in per_rank],
                "wire_GBps": round(wire * world * args.steps / wall_max / 1e9, 2),
                "kernel_ms": round(kern_max, 4),
                # the timed launches' spread (rank 0): the mean above averages the chip's clock transient over the
                # first launches of a run (profiles/r05_transient.txt); median and minimum beside it, nothing hidden
                "kernel_ms_median": round(float(np.median(kern_each)), 4),
                "kernel_ms_min": round(float(np.min(kern_each)), 4),
                "kernel_ms_max": round(float(np.max(kern_each)), 4),
                "step_kernel_ms": round(step_ms, 4),
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
                "traffic_source": traffic_note,
                "algorithmic_read_bytes": read_bytes,
                "record_write_bytes": write_bytes,
                # the kernel also writes its records: algorithmic read + record bytes over the same launch time (the
                # kernel's total algorithmic traffic against the same peak; `frac` above is the read side alone)
                "rw_achieved": round((read_bytes + write_bytes) / (kern_ms * 1e-3) / 1e9, 1),
                "rw_frac": round((read_bytes + write_bytes) / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            },
            "cpu_baseline": cpu,
        }
        if e2e is not None:
            line["e2e_host_to_host"] = e2e
        if flow_check is not None:
            line["config"]["flow_table"] = flow_check
        if keys_equal is not None:
            line["config"]["flow_keys_equal_hash5"] = keys_equal
        if brief_equal is not None:
            line["config"]["brief_equal_summary_half"] = brief_equal
        if stats_line is not None:
            line["config"]["collect_stats"] = stats_line
        if tuple_check is not None:
            line["config"]["tuples"] = tuple_check
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
