"""bench.py's own N-GPU launch (no external launcher), on CPU.

`python bench.py --gpus N` must run N ranks itself — a child `torch.distributed.run` started before anything
touches the GPU — and a rank must refuse to run when WORLD_SIZE differs from --gpus, so a line's n_gpus is
always the GPU count that was asked for. Mirrors the reference's self-contained one-worker-per-core launch
(Pcap++/src/DpdkDeviceList.cpp:346-440, Examples/DpdkExample-FilterTraffic/main.cpp:279-287).
"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def test_launcher_command_line():
    argv = ["--gpus", "8", "--config", "4", "--steps", "3"]
    cmd = bench.launcher_cmd(8, argv, 29555)
    assert cmd[0] == sys.executable
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(str((ROOT / "bench.py").resolve()))
    assert cmd[i + 1:] == argv  # the ranks get the same arguments


def test_check_world():
    assert bench.check_world(1, {}) is None                      # plain 1-GPU run
    assert bench.check_world(4, {}) == 0                         # parent: launch 4 ranks
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) is None     # a rank of the 4-rank job
    assert bench.check_world(1, {"WORLD_SIZE": "1"}) is None
    assert bench.check_world(8, {"WORLD_SIZE": "2"}) == 2        # mismatch
    assert bench.check_world(1, {"WORLD_SIZE": "8"}) == 2


def test_world_mismatch_exits_nonzero_before_gpu():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr and r.stdout == ""


def test_parent_forwards_rank_output_and_exit_code(tmp_path):
    """launch_ranks streams the child's stdout and returns its exit code (child stubbed by a tiny script)."""
    fake = tmp_path / "fake_rank.py"
    fake.write_text("import sys\nprint('{\"n_gpus\": 2}')\nsys.exit(3)\n")
    r = subprocess.run([sys.executable, "-c",
                        "import sys; sys.path.insert(0, %r); import bench; "
                        "bench.launcher_cmd = lambda g, a, p: [sys.executable, %r]; "
                        "sys.exit(bench.launch_ranks(2, []))" % (str(ROOT), str(fake))],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 3
    assert r.stdout.strip() == '{"n_gpus": 2}'


def test_real_launcher_starts_n_ranks(tmp_path):
    """The exact torch.distributed.run command line bench.py builds starts N ranks with WORLD_SIZE = N (a stub rank
    script in place of bench.py; gloo rendezvous over 127.0.0.1, no GPU)."""
    stub = tmp_path / "rank.py"
    stub.write_text("import os, sys\n"
                    "import torch.distributed as dist\n"
                    "dist.init_process_group('gloo')\n"
                    "ws = dist.get_world_size()\n"
                    "dist.barrier()\n"
                    "if dist.get_rank() == 0:\n"
                    "    print('ranks', ws, os.environ['WORLD_SIZE'], ' '.join(sys.argv[1:]), flush=True)\n"
                    "dist.destroy_process_group()\n")
    cmd = bench.launcher_cmd(2, ["--config", "4"], bench.free_port())
    cmd[cmd.index(str((ROOT / "bench.py").resolve()))] = str(stub)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ranks 2 2 --config 4" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_bench_small_run_checks_its_records(cfg):
    """bench.py end to end on the GPU at a small size for the configs whose launch differs from the default one: config 2
    (5-tuple extract alone, SHORT window), config 4 (dense keys + collectStats without a summary, SHORT window, the flow
    table) and config 5 (two-round window, the brief + PACKED rows) -- one JSON line whose own checks hold."""
    import json

    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--config", str(cfg), "--packets", "200000", "--steps",
                        "3", "--warmup", "1", "--no-cpu-baseline", "--no-e2e", "--no-traffic"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    c = line["config"]
    assert line["n_gpus"] == 1 and line["value"] > 0 and c["flagged_packets"] == 0
    if cfg == 2:
        assert c["records"] == "tuples" and c["window"] == "short"
        assert c["tuples"] == {"with_5tuple": 200000, "hash5_equal_summary": True}
    if cfg == 4:
        assert c["records"] == "keys" and c["window"] == "short" and c["flow_keys_equal_hash5"]
        assert c["flow_table"]["exact"] and c["flow_table"]["conserved"] and c["collect_stats"]["consistent"]
    if cfg == 5:
        assert c["records"] == "brief" and c["layout"] == "packed" and c["window"] == "default"
        assert c["brief_equal_summary_half"]


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,cfg", [(2, 4), (2, 3), (8, 4), (8, 3)], ids=["n2-cfg4", "n2-cfg3", "n8-cfg4", "n8-cfg3"])
def test_bench_ranks_self_launch(ranks, cfg, tmp_path):
    """`bench.py --gpus N` through its own launch (a child torch.distributed.run, N ranks over gloo sharing the box's
    one card: a code-path check of the N>1 path -- the shard ranges, seeds and the host merge of N tables the driver's
    8-GPU run uses -- not a scaling number): one line from rank 0 with n_gpus N and every rank's times; config 4 merges
    the N ranks' flow tables exactly with every packet conserved and sums their collectStats, and the merged table
    equals a single-pass host group-by of the restatement's hash5Tuple over the stream's first N shards; the line
    carries rank 0's CPU baseline (measured after the timed region)."""
    import json

    npk = 200_000 if ranks == 2 else 100_000
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    dump = tmp_path / "flows.npz"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(ranks), "--dist-backend", "gloo",
                        "--config", str(cfg), "--packets", str(npk), "--steps", "3", "--warmup", "1", "--no-e2e",
                        "--no-traffic", "--cpu-sample", "20000", "--cpu-seconds", "0.5", "--dump-flows", str(dump)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    c = line["config"]
    assert line["n_gpus"] == ranks and c["ranks"] == ranks and c["dist_backend"] == "gloo"
    assert c["parallelism"] == f"shard{ranks} (no collective)"
    assert len(c["per_rank_kernel_ms"]) == ranks and all(t > 0 for t in c["per_rank_kernel_ms"])
    assert len(c["per_rank_wall_ms_per_step"]) == ranks
    assert line["value"] > 0 and c["flagged_packets"] == 0
    assert line["cpu_baseline"] is not None and line["cpu_baseline"]["value"] > 0
    if cfg == 4:
        ft = c["flow_table"]
        assert ft["ranks_merged"] == ranks and ft["exact"] and ft["conserved"]
        assert ft["packets_counted"] == ft["expected"] == ranks * npk * 4
        assert ft["merged_within_universe"] and ft["flows_spanning_ranks"] > 0
        assert len(ft["per_rank_flows"]) == ranks
        cs = c["collect_stats"]
        assert cs["consistent"] and cs["ranks_merged"] == ranks and cs["packet_count"] == ranks * npk
        # the merged table equals a single-pass map over the union of the N shards (the stream's first N * npk
        # packets), key for key: the restatement's hash5Tuple grouped on the host, times the 4 launches per rank
        import numpy as np

        import oracle
        from pcapplusplus_amd import abi, shard, synth

        m = np.load(dump)
        whole = synth.flow_stream(0, ranks * npk, 4, flows=bench.CONFIG4_FLOWS)
        s, _ = oracle.oracle_parse(whole, abi.make_opts(0, 8, False, 0), threads=8)
        want = shard.flow_table(s["hash5"], whole.caplens)
        launches = int(m["launches"][0])
        got = {int(k): (int(p) // launches, int(b) // launches) for k, p, b in zip(m["keys"], m["packets"], m["bytes"])}
        assert all(int(p) % launches == 0 for p in m["packets"])
        if m["key0"][0]:
            got[-1] = (int(m["key0"][0]) // launches, int(m["key0"][1]) // launches)
        assert got == want and int(m["key0"][2]) == 0
