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

STUB = r'''
import json, os, sys, time
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
mode = sys.argv[1]
if mode == "fail" and rank == 1:
    sys.exit(3)
if mode == "fail":
    time.sleep(600)                  # a peer blocked forever (e.g. in a collective)
import torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(rank + 1)])
dist.all_reduce(t)
print(f"rank {rank} says hello")     # non-zero ranks: must not reach the forwarded stdout
if rank == 0:
    print(json.dumps({"n_gpus": world, "sum": t.item(), "local": int(os.environ["LOCAL_RANK"]),
                      "addr": os.environ["MASTER_ADDR"]}))
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
    rc = bench.spawn_ranks(3, [sys.executable, stub, "ok"], env=env, out=out)
    assert rc == 0
    lines = [ln for ln in out.getvalue().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    j = json.loads(lines[0])
    assert j == {"n_gpus": 3, "sum": 6.0, "local": 0, "addr": "127.0.0.1"}
    assert "rank 1 says hello" not in out.getvalue() and "rank 2 says hello" not in out.getvalue()


def test_spawn_ranks_fails_when_a_rank_fails(stub):
    out = io.StringIO()
    rc = bench.spawn_ranks(3, [sys.executable, stub, "fail"], out=out, grace_s=1.0)
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
