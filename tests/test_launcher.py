"""CPU tests of bench.py's multi-rank launcher: with
--gpus N > 1 and no WORLD_SIZE the bench starts N ranks itself through
torch.distributed.run (a child process, no exec), every rank sees
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, rank 0's JSON line is relayed and a
failing rank fails the launch.  Ranks here run a stand-in script on gloo."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

RANK_SCRIPT = r'''
import json, os, sys
import torch, torch.distributed as dist
env = {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
dist.init_process_group("gloo")
t = torch.tensor([float(int(env["RANK"]) + 1)])
dist.all_reduce(t)
if "--fail-rank" in sys.argv and int(env["RANK"]) == int(sys.argv[sys.argv.index("--fail-rank") + 1]):
    sys.exit(3)
ranks = [None] * dist.get_world_size()
dist.all_gather_object(ranks, env)
if dist.get_rank() == 0:
    print("some log line", flush=True)
    print(json.dumps({"metric": "m", "n_gpus": dist.get_world_size(), "sum": t.item(), "envs": ranks,
                      "argv": sys.argv[1:]}), flush=True)
dist.destroy_process_group()
'''


@pytest.fixture
def rank_script(tmp_path, monkeypatch):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    monkeypatch.setenv("IWAE_DIST_BACKEND", "gloo")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    return str(p)


def test_launcher_command_shape():
    cmd = bench.launcher_command(4, ["--gpus", "4", "--steps", "7"], 29555, "/x/bench.py")
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-5:] == ["/x/bench.py", "--gpus", "4", "--steps", "7"]


def test_check_world_refuses_more_ranks_than_gpus_under_rccl():
    with pytest.raises(SystemExit, match="needs 8 visible GPUs"):
        bench.check_world(8, "nccl", 1)
    bench.check_world(8, "nccl", 8)
    bench.check_world(8, "gloo", 1)          # rehearsal: ranks may share a GPU
    with pytest.raises(SystemExit):
        bench.check_world(0, "gloo", 1)


def test_launch_ranks_relays_rank0_line(rank_script, capfd):
    rc = bench.launch_ranks(2, ["--gpus", "2", "--steps", "3"], script=rank_script)
    out, err = capfd.readouterr()
    assert rc == 0
    lines = [l for l in out.splitlines() if l.strip()]
    assert len(lines) == 1, out                 # only the JSON line reaches stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["sum"] == 3.0
    assert sorted(int(e["RANK"]) for e in rec["envs"]) == [0, 1]
    assert sorted(int(e["LOCAL_RANK"]) for e in rec["envs"]) == [0, 1]
    assert all(e["WORLD_SIZE"] == "2" and e["MASTER_ADDR"] == "127.0.0.1" for e in rec["envs"])
    assert rec["argv"] == ["--gpus", "2", "--steps", "3"]
    assert "some log line" in err


def test_launch_ranks_fails_when_a_rank_fails(rank_script, capfd):
    rc = bench.launch_ranks(2, ["--fail-rank", "1"], script=rank_script)
    out, _ = capfd.readouterr()
    assert rc != 0
    assert out.strip() == ""


def test_bench_refuses_rccl_world_beyond_visible_gpus(monkeypatch):
    monkeypatch.delenv("IWAE_DIST_BACKEND", raising=False)
    monkeypatch.setattr(bench, "visible_gpus", lambda: 1)
    with pytest.raises(SystemExit, match="needs 2 visible GPUs"):
        bench.launch_ranks(2, ["--gpus", "2"])
