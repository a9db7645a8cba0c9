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
