"""bench.py --gpus N launches its own ranks (the driver's N-GPU form without torch.distributed.run around it)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_launcher_command_is_one_rank_per_gpu_on_this_node():
    cmd = bench.launcher_command(["--gpus", "8", "--steps", "5", "--warmup", "1"], 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5", "--warmup", "1"]


def test_free_port_is_bindable():
    import socket
    p = bench.free_port()
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", p))


def test_more_gpus_than_devices_fails_under_nccl():
    """No GPU here: --gpus 2 under the nccl backend must refuse before starting any rank (exit 2)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["EPIPF_DIST_BACKEND"] = "nccl"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s)" in r.stderr


def test_gpus_defaults_to_the_launchers_world_size():
    """Under an external launcher (torchrun --nproc-per-node N bench.py) --gpus may be omitted: it becomes the world
    size; without a launcher it is 1; an explicit --gpus that contradicts WORLD_SIZE is refused."""
    import argparse
    a = argparse.Namespace(gpus=None)
    assert bench.resolve_gpus(a, {"WORLD_SIZE": "4"}) is None and a.gpus == 4
    a = argparse.Namespace(gpus=None)
    assert bench.resolve_gpus(a, {}) is None and a.gpus == 1
    a = argparse.Namespace(gpus=4)
    assert bench.resolve_gpus(a, {"WORLD_SIZE": "4"}) is None
    a = argparse.Namespace(gpus=2)
    assert "WORLD_SIZE=4 but --gpus 2" in bench.resolve_gpus(a, {"WORLD_SIZE": "4"})


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


@pytest.mark.gpu
def test_bench_launches_two_gloo_ranks_itself():
    """One-box rehearsal of the self-launch: two ranks (gloo, sharing GPU 0) started by bench.py, one JSON line."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["EPIPF_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--chains", "4", "--config", "1", "--no-cpu-baseline", "--configs", "none"], env=env,
                       capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "launching 2 ranks" in r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    assert lines[0]["ranks"] == 2 and len(lines[0]["rank_devices"]) == 2
    assert lines[0]["gathered_draws_shape"][0] == 8


@pytest.mark.gpu
def test_bench_north_star_layout_four_gloo_ranks():
    """BASELINE config 5's layout -- one chain per GPU, the lane-group kernel -- through the multi-rank path: four gloo
    ranks sharing GPU 0, each one chain of the 2-group model; the draws of all four are gathered."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["EPIPF_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--config", "5", "--chains", "1",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--configs", "none"], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "launching 4 ranks" in r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["ranks"] == 4 and len(d["rank_devices"]) == 4
    assert d["gathered_draws_shape"][0] == 4
    assert d["lanes_per_particle"] > 1 and d["roofline"]["kernel"].startswith("pf_step_group_kernel")
    assert d["config"]["chains_per_gpu"] == 1 and d["proposal"]["h"] == 1.0
