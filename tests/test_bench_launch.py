"""bench.py's rank launcher on the CPU (no GPU call): `--gpus N` without torchrun
starts N ranks itself through torch.distributed.run, and a rank whose WORLD_SIZE
differs from --gpus refuses to run (--gpus was a no-op)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=e, capture_output=True, text=True,
                          timeout=300)


def test_gpus_n_launches_n_ranks():
    r = _bench(["--gpus", "3", "--launch-probe"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1, 2]
    assert {d["world"] for d in lines} == {3}
    assert sorted(d["local_rank"] for d in lines) == [0, 1, 2]


def test_force_dist_launches_one_rank():
    r = _bench(["--gpus", "1", "--force-dist", "--launch-probe"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"rank": 0, "world": 1, "local_rank": 0}]


def test_world_size_mismatch_is_an_error():
    r = _bench(["--gpus", "4", "--launch-probe"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_launch_cmd_shape():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launch_cmd(["--gpus", "8", "--steps", "5"], 8, 29500)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
