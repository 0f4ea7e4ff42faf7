"""bench.py's multi-process paths on the CPU (gloo, world size 2): the self-spawning launcher
(``bench.py --gpus N`` outside torchrun) and the torchrun launch the driver uses.  Both must print
exactly one JSON line, from rank 0, with n_gpus = the world size the process group saw."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def _check(r, world):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    res = lines[0]
    assert res["n_gpus"] == world and res["config"]["world_size_seen"] == world
    assert res["steps"] == 3 and res["value"] > 0 and res["scaling"] == "weak"
    assert res["config"]["global_batch"] == world * res["config"]["batch_per_gpu"]


ARGS = ["--device", "cpu", "--workload", "selftest", "--steps", "3", "--warmup", "1"]


@pytest.mark.parametrize("world", [1, 2])
def test_self_spawning_launcher(world):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(world)] + ARGS,
                       capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    _check(r, world)


def test_torchrun_launch():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        os.path.join(REPO, "bench.py"), "--gpus", "2"] + ARGS,
                       capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    _check(r, 2)


def test_cpu_device_is_selftest_only():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--device", "cpu", "--workload", "lipsync"],
                       capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode != 0 and "selftest" in (r.stderr + r.stdout)
