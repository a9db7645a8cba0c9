"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"` runs here (no GPU): the oracle against the reference's golden records and KATs, host
logic, and the C-ABI library's exported symbols. `-m gpu` runs on an MI355X: HIP engine parity.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP engine runs)")


def make_examples():
    """`make -C examples` under an exclusive lock: xdist workers of test_facade and test_examples build the same
    binaries, and an unlocked concurrent rebuild leaves one worker running a half-written executable."""
    import fcntl
    import subprocess

    root = Path(__file__).resolve().parents[1]
    (root / "examples" / "bin").mkdir(exist_ok=True)
    with open(root / "examples" / "bin" / ".build.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        return subprocess.run(["make", "-s", "-C", str(root / "examples")], capture_output=True, text=True)


def golden_files():
    return sorted(GOLDEN.glob("*.npz"))


def load_golden(path: Path):
    """(PacketBatch, {variant: (opts, sum, lay)}) from a tests/golden/*.npz fixture."""
    from pcapplusplus_amd import abi
    from pcapplusplus_amd.pcap import PacketBatch

    z = np.load(path, allow_pickle=False)
    b = PacketBatch(z["data"], z["offsets"], z["caplens"], int(z["linktype"]))
    b.meta["set_names"] = list(z["set_names"])
    b.meta["set_index"] = z["set_index"]
    variants = {}
    for key in z.files:
        if key.startswith("opts_"):
            v = key[5:]
            fam, osi, cs, ml = (int(x) for x in z[key])
            variants[v] = (abi.make_opts(fam, osi, bool(cs), ml), z[f"sum_{v}"], z[f"lay_{v}"])
    return b, variants


@pytest.fixture(scope="session")
def engine():
    """The HIP engine on cuda:0 (gpu tests only)."""
    from pcapplusplus_amd.engine import Engine

    eng = Engine(0)
    yield eng
    eng.close()
