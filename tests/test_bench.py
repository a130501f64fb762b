"""bench.py's contract line, in both multi-GPU drivers' shapes (small workloads).

The single-process mode (--devices, rt_render_multi: the north_star's Go-host path) is
rehearsed on one GPU with two shares on device 0; torchrun's one-process-per-GPU mode
needs distinct GPUs (RCCL) and is covered by tests/test_distributed.py with gloo.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--scene", "cornell", "--width", "160", "--spp", "64", "--steps", "2", "--warmup", "1",
         "--no-cpu-baseline", "--no-extra-configs"]


def _bench(*args):
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *SMALL, *args],
                       capture_output=True, text=True, timeout=300, cwd=REPO)
    return p


def test_devices_mode_rejects_mismatched_count():
    p = _bench("--gpus", "3", "--devices", "0,0")
    assert p.returncode != 0 and "--devices must list --gpus devices" in p.stderr


@pytest.mark.gpu
def test_devices_mode_line(gpu):
    p = _bench("--gpus", "2", "--devices", "0,0")
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1  # distinct devices: both shares ran on device 0
    assert "rt_render_multi" in line["config"]["parallelism"]
    assert line["value"] > 0 and line["steps"] == 2
    assert line["roofline"]["launches"] == 2


@pytest.mark.gpu
def test_devices_mode_rccl_gather_line(gpu):
    """--gather rccl: the shares collected by one ncclGather (RT_FLAG_GATHER_RCCL); on a
    one-GPU box the device list is [0] (RCCL needs distinct devices)."""
    p = _bench("--gpus", "1", "--devices", "0", "--gather", "rccl")
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert "rccl gather" in line["config"]["parallelism"]
    assert line["value"] > 0 and line["steps"] == 2


def test_gather_option_rejects_unknown():
    p = _bench("--gather", "nccl-allgather")
    assert p.returncode != 0 and "invalid choice" in p.stderr


@pytest.mark.gpu
def test_multi_device_check_child_mode(gpu):
    """bench.py's distinct-device check (run by rank 0 of a torchrun job on a multi-GPU
    node) in its child-process mode; on one GPU the device list is [0]."""
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--multi-device-check",
                        "1"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["devices"] == [0]
    for k in ("peer", "peer_reversed", "rccl"):
        assert res[k]["bitwise"], res
