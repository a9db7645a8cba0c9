"""N>1 path on CPU: world_size-2 gloo process group. Each rank parses its contiguous shard (with the
restatement — the device path is covered by -m gpu), builds its flow table, and the host merge equals a
single-pass table; the bench's max-over-ranks timing reduction works across ranks."""
from __future__ import annotations

import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from pcapplusplus_amd import shard


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank: int, world: int, port: int, q):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import torch

    import oracle
    from pcapplusplus_amd import abi, synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = synth.config(4, 20_000)
    lo, hi = shard.shard_range(b.n, world, rank)
    part = b.slice(lo, hi)
    s, _ = oracle.oracle_parse(part, abi.make_opts(0, 8, False, 0))
    table = shard.flow_table(s["hash5"], part.caplens)
    tables = [None] * world
    dist.all_gather_object(tables, table)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        full, _ = oracle.oracle_parse(b, abi.make_opts(0, 8, False, 0))
        q.put((shard.merge_flow_tables(tables) == shard.flow_table(full["hash5"], b.caplens), float(t[0])))
    dist.destroy_process_group()


def test_two_rank_shards_merge_to_single_pass():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    equal, tmax = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert equal
    assert tmax == 2.0


def _device_format(hash5: np.ndarray, caplens: np.ndarray, capacity: int):
    """The table pcppx_flow_count_device would hold for these packets (any slot order): keys u32[capacity] with
    zeros for empty slots, packets / bytes u64[capacity], stats u64[4] (key-0 packets / bytes, drops)."""
    t = shard.flow_table(hash5, caplens)
    keys = np.zeros(capacity, np.uint32)
    pk = np.zeros(capacity, np.uint64)
    by = np.zeros(capacity, np.uint64)
    stats = np.zeros(4, np.uint64)
    rng = np.random.default_rng(len(t))
    slots = rng.permutation(capacity)
    j = 0
    for k, (p, b) in t.items():
        if k == -1:
            stats[0], stats[1] = p, b
            continue
        keys[slots[j]], pk[slots[j]], by[slots[j]] = k, p, b
        j += 1
    return keys, pk, by, stats


def _device_worker(rank: int, world: int, port: int, q):
    """Each rank holds a device-format flow table of its contiguous shard of the one config-4 stream; rank 0 merges the
    compact tables (the bench's config-4 host merge) and compares with one table over the union of the shards, key for
    key; flows span the shards (the merge adds real counts)."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

    import oracle
    from pcapplusplus_amd import abi, synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # bench.py's config-4 layout: rank r parses packets [n r, n (r+1)) of ONE stream over ONE flow universe
    n = 30_000
    part = synth.flow_stream(n * rank, n * (rank + 1), 4, flows=3000)
    s, _ = oracle.oracle_parse(part, abi.make_opts(0, 8, False, 0))
    mine = shard.compact_device_table(*_device_format(s["hash5"], part.caplens, 1 << 13))
    tables = [None] * world
    dist.all_gather_object(tables, mine)
    if rank == 0:
        merged = shard.merge_device_tables(tables)
        # the single-pass map over the union of the shards: the stream's first n * world packets in one batch
        whole = synth.flow_stream(0, n * world, 4, flows=3000)
        full, _ = oracle.oracle_parse(whole, abi.make_opts(0, 8, False, 0))
        counted = int(merged["packets"].sum()) + merged["key0_packets"] + merged["dropped"]
        spanning = sum(len(t["keys"]) for t in tables) - len(merged["keys"])
        q.put((shard.merged_to_dict(merged) == shard.flow_table(full["hash5"], whole.caplens),
               counted == whole.n and spanning > 100))
    dist.destroy_process_group()


def test_two_rank_device_tables_merge_to_single_pass():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_device_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    equal, conserved = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert equal and conserved


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 100, 12_500_001):
        for world in (1, 2, 3, 8):
            r = [shard.shard_range(n, world, k) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))
            assert max(h - l for l, h in r) - min(h - l for l, h in r) <= 1


def test_flow_table_merge_is_key_sum():
    h = np.array([5, 0, 5, 7, 0], np.uint32)
    c = np.array([10, 20, 30, 40, 50], np.uint32)
    t = shard.flow_table(h, c)
    assert t == {5: (2, 40), 7: (1, 40), -1: (2, 70)}
    assert shard.merge_flow_tables([t, t]) == {5: (4, 80), 7: (2, 80), -1: (4, 140)}
