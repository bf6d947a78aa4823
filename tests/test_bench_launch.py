"""CPU: `bench.py --gpus N` starting its own N ranks (spawn_ranks) and the launcher check
(world_from_env), with a stub worker in place of the GPU bench: the ranks get the
torch.distributed.run environment (a real gloo all_reduce over it), rank 0's JSON line is
forwarded, and a failing rank makes the launch fail without leaving its peers behind."""
import io
import json
import os
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = r'''
import json, os, sys, time
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
mode = sys.argv[1]
if mode == "fail" and rank == 1:
    sys.exit(3)
if mode == "fail":
    time.sleep(600)                  # a peer blocked forever (e.g. in a collective)
import torch, torch.distributed as dist
sys.path.insert(0, sys.argv[2])
import bench
dist.init_process_group("gloo")
t = torch.tensor([float(rank + 1)])
dist.all_reduce(t)
print(f"rank {rank} says hello")     # non-zero ranks: must not reach the forwarded stdout
probe = {"k2_ms": [1.7 + rank, 1.9 + rank], "k2_ms_chosen": 1.7 + rank, "k2_ms_median_unprobed": 1.8 + rank}
per_rank = bench.gather_per_rank(dist, rank, bench.rank_record(rank, int(os.environ["LOCAL_RANK"]),
                                                                [0.5, 1.7 + rank, 0.3, 0.01], probe, 0.05 * (rank + 1)))
if rank == 0:
    print(json.dumps({"n_gpus": world, "sum": t.item(), "local": int(os.environ["LOCAL_RANK"]),
                      "addr": os.environ["MASTER_ADDR"], "per_rank": per_rank}))
else:
    assert per_rank is None
dist.destroy_process_group()
'''


@pytest.fixture()
def stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return str(p)


def test_spawn_ranks_forwards_rank0_json(stub):
    out = io.StringIO()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rc = bench.spawn_ranks(3, [sys.executable, stub, "ok", ROOT], env=env, out=out)
    assert rc == 0
    lines = [ln for ln in out.getvalue().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    j = json.loads(lines[0])
    per_rank = j.pop("per_rank")
    assert j == {"n_gpus": 3, "sum": 6.0, "local": 0, "addr": "127.0.0.1"}
    # every rank's own K2 time, probe and spread on rank 0's line, in rank order
    assert [r["rank"] for r in per_rank] == [0, 1, 2] and [r["local_rank"] for r in per_rank] == [0, 1, 2]
    assert [r["quantize_ms"] for r in per_rank] == [1.7, 2.7, 3.7]
    assert [r["quantize_ms_median_unprobed"] for r in per_rank] == [1.8, 2.8, 3.8]
    assert all(r["probe_spread_ms"] == 0.2 for r in per_rank)
    assert [r["elapsed_s"] for r in per_rank] == [0.05, 0.1, 0.15]
    assert "rank 1 says hello" not in out.getvalue() and "rank 2 says hello" not in out.getvalue()


def test_spawn_ranks_fails_when_a_rank_fails(stub):
    out = io.StringIO()
    rc = bench.spawn_ranks(3, [sys.executable, stub, "fail", ROOT], out=out, grace_s=1.0)
    assert rc == 1


def test_world_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    args = bench.parse(["--gpus", "8"])
    with pytest.raises(SystemExit):
        bench.world_from_env(args)
    args = bench.parse([])
    assert bench.world_from_env(args) == 2 and args.gpus == 2
    monkeypatch.delenv("WORLD_SIZE")
    args = bench.parse([])
    assert bench.world_from_env(args) == 1 and args.gpus == 1
