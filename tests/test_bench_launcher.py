"""bench.py's multi-GPU launcher (CPU): `--gpus N` outside torchrun starts one process per GPU through
torch.distributed.run before anything touches the GPU; under torchrun the real world size is used."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_needs_launch():
    assert not bench.needs_launch(1, {})
    assert bench.needs_launch(2, {})
    assert not bench.needs_launch(8, {"WORLD_SIZE": "8"})


def test_launch_cmd():
    cmd = bench.launch_cmd(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_world_size_check():
    bench.world_size_check(1, 8)
    bench.world_size_check(8, 8)
    with pytest.raises(SystemExit):
        bench.world_size_check(4, 8)


def test_relaunch_spawns_one_process_per_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-launch"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 for d in lines)
    assert sorted(d["local_rank"] for d in lines) == [0, 1]
