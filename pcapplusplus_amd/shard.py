"""Multi-GPU sharding helpers: packets are independent, so every GPU takes its own
contiguous shard and nothing crosses GPUs on the data path. Per-GPU flow tables are merged on the
host by key, as DpdkExample-FilterTraffic sums its per-core tables at exit
(Examples/DpdkExample-FilterTraffic/main.cpp:279-287)."""
from __future__ import annotations

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) packet range of `rank` for a fixed total (strong-scaling layout)."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_seed(config_seed: int, rank: int) -> int:
    """Seed of a rank's own synthetic shard (weak-scaling layout: fixed work per GPU)."""
    return config_seed + 1000 * rank


def flow_table(hash5: np.ndarray, caplens: np.ndarray) -> dict[int, tuple[int, int]]:
    """{flow key: (packets, bytes)} for non-zero keys; key 0 (non-5-tuple packets,
    PacketUtils.cpp:141-148) is returned under -1 so it can be merged like the others."""
    keys, inv = np.unique(hash5, return_inverse=True)
    pk = np.bincount(inv)
    by = np.bincount(inv, weights=caplens.astype(np.float64)).astype(np.int64)
    return {(int(k) if k != 0 else -1): (int(p), int(b)) for k, p, b in zip(keys, pk, by)}


def merge_flow_tables(tables: list[dict[int, tuple[int, int]]]) -> dict[int, tuple[int, int]]:
    out: dict[int, tuple[int, int]] = {}
    for t in tables:
        for k, (p, b) in t.items():
            q = out.get(k, (0, 0))
            out[k] = (q[0] + p, q[1] + b)
    return out


def device_table_to_dict(keys: np.ndarray, packets: np.ndarray, bytes_: np.ndarray,
                         stats: np.ndarray) -> dict[int, tuple[int, int]]:
    """A pcppx_flow_count_device table (keys/packets/bytes arrays + stats) as a flow_table() dict."""
    used = keys != 0
    out = {int(k): (int(p), int(b)) for k, p, b in zip(keys[used], packets[used], bytes_[used])}
    if stats[0]:
        out[-1] = (int(stats[0]), int(stats[1]))
    return out


def compact_device_table(keys: np.ndarray, packets: np.ndarray, bytes_: np.ndarray, stats: np.ndarray) -> dict:
    """The used slots of a pcppx_flow_count_device table (keys u32[capacity], zero = empty; packets / bytes
    u64[capacity]; stats u64[>=3]: key-0 packets / bytes, packets that found no free slot) as compact arrays, the
    unit a rank ships to the merging host."""
    keys = keys.view(np.uint32)
    used = keys != 0
    return {"keys": keys[used].copy(), "packets": packets.view(np.uint64)[used].copy(),
            "bytes": bytes_.view(np.uint64)[used].copy(), "stats": stats.view(np.uint64)[:3].copy()}


def merge_device_tables(tables: list[dict]) -> dict:
    """Merge per-GPU device flow tables by key (vectorised), as FilterTraffic sums its per-core tables at exit
    (Examples/DpdkExample-FilterTraffic/main.cpp:279-287): {keys, packets, bytes} sorted by key, plus the summed
    key-0 bucket and no-free-slot count."""
    if not tables:
        return {"keys": np.zeros(0, np.uint32), "packets": np.zeros(0, np.uint64), "bytes": np.zeros(0, np.uint64),
                "key0_packets": 0, "key0_bytes": 0, "dropped": 0}
    k = np.concatenate([t["keys"] for t in tables])
    uk, inv = np.unique(k, return_inverse=True)
    pk = np.zeros(len(uk), np.uint64)
    by = np.zeros(len(uk), np.uint64)
    np.add.at(pk, inv, np.concatenate([t["packets"] for t in tables]))
    np.add.at(by, inv, np.concatenate([t["bytes"] for t in tables]))
    st = np.sum([t["stats"].astype(np.uint64) for t in tables], axis=0)
    return {"keys": uk, "packets": pk, "bytes": by, "key0_packets": int(st[0]), "key0_bytes": int(st[1]),
            "dropped": int(st[2])}


def merged_to_dict(m: dict) -> dict[int, tuple[int, int]]:
    """A merge_device_tables() result in flow_table() form (key 0 under -1)."""
    out = {int(k): (int(p), int(b)) for k, p, b in zip(m["keys"], m["packets"], m["bytes"])}
    if m["key0_packets"]:
        out[-1] = (m["key0_packets"], m["key0_bytes"])
    return out
