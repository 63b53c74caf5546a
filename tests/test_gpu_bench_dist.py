"""bench.py's multi-rank branch (BASELINE config 4) exercised before the
driver's 8-GPU scaling run: two ranks launched by torch.distributed.run on the one
GPU of the test box (--same-device, gloo for the record all-gather), strong scaling
over one list of frames. The all-gathered per-frame box records must equal a
single-rank run over the same list (fp32: per-frame results do not depend on the
batch a frame lands in)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--scaling", "strong", "--frames", "6", "--batch", "6", "--steps", "1", "--warmup", "0", "--no-timing",
          "--compare", "", "--host-pipeline", "0", "--no-cpu-baseline"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, out):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd + ["--records-out", out], cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


@pytest.mark.parametrize("frames,batch", [(6, 6), (13, 4)])
def test_bench_two_ranks_strong_equals_single_rank(gpu, tmp_path, frames, batch):
    """(13, 4): shards of 7 / 6 frames in batches of 4 through vdmi.dist.process_frames
    (a short last batch on each rank, records padded to 7 rows)."""
    from vdmi.dist import unpack_records
    one = str(tmp_path / "one.npy")
    two = str(tmp_path / "two.npy")
    common = list(COMMON)
    common[common.index("--frames") + 1] = str(frames)
    common[common.index("--batch") + 1] = str(batch)
    _run([sys.executable, "bench.py"] + common, one)
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                "--backend", "gloo", "--same-device"] + common, two)
    assert '"n_gpus": 2' in out
    r1, r2 = unpack_records(np.load(one)), unpack_records(np.load(two))
    assert list(r1) == list(range(frames)) and list(r2) == list(range(frames))
    assert sum(v[3] for v in r1.values()) > 0
    assert r2 == r1


def test_bench_self_launch_two_ranks_equals_single_rank(gpu, tmp_path):
    """`python bench.py --gpus 2` with no torchrun around it starts both ranks itself."""
    from vdmi.dist import unpack_records
    one = str(tmp_path / "one.npy")
    two = str(tmp_path / "two.npy")
    _run([sys.executable, "bench.py"] + COMMON, one)
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", "--same-device"] + COMMON, two)
    assert '"n_gpus": 2' in out and "gloo all-gather" in out
    r1, r2 = unpack_records(np.load(one)), unpack_records(np.load(two))
    assert list(r2) == list(range(6)) and sum(v[3] for v in r1.values()) > 0
    assert r2 == r1


def test_bench_rccl_world1_equals_no_dist(gpu, tmp_path):
    """The nccl (= RCCL) branch of bench.py -- init_process_group("nccl", device_id=...)
    and all_gather_into_tensor of the box records on the device -- at one rank: the
    gathered records equal the no-dist run's."""
    from vdmi.dist import unpack_records
    one = str(tmp_path / "one.npy")
    rc = str(tmp_path / "rccl.npy")
    _run([sys.executable, "bench.py"] + COMMON, one)
    out = _run([sys.executable, "bench.py", "--gpus", "1", "--force-dist", "--backend", "nccl"] + COMMON, rc)
    assert '"n_gpus": 1' in out and "RCCL all-gather" in out
    r1, r2 = unpack_records(np.load(one)), unpack_records(np.load(rc))
    assert list(r2) == list(range(6)) and sum(v[3] for v in r1.values()) > 0
    assert r2 == r1


@pytest.mark.parametrize("dist", [False, True])
def test_bench_inflight_records_equal_single_slot(gpu, tmp_path, dist):
    """bench.py --inflight 2 (two contexts taking consecutive steps on their own streams;
    the records of a step are packed, and with --force-dist all-gathered over RCCL, on
    that step's stream): the last step's records (slot 1's) equal a one-slot run's."""
    from vdmi.dist import unpack_records
    one = str(tmp_path / "one.npy")
    two = str(tmp_path / "two.npy")
    common = [c if c != "1" or i != COMMON.index("--steps") + 1 else "2" for i, c in enumerate(COMMON)]
    extra = ["--gpus", "1", "--force-dist", "--backend", "nccl"] if dist else []
    _run([sys.executable, "bench.py"] + extra + common, one)
    out = _run([sys.executable, "bench.py", "--inflight", "2"] + extra + common, two)
    assert '"batches_in_flight": 2' in out
    r1, r2 = unpack_records(np.load(one)), unpack_records(np.load(two))
    assert list(r2) == list(range(6)) and sum(v[3] for v in r1.values()) > 0
    assert r2 == r1
