"""bench.py --gpus N launches N ranks itself (the driver's scaling command is `python bench.py
--gpus N`): one torch.distributed.run child, one rank per GPU, never a re-exec.
CPU only: the ranks run with --rank-probe, which reports the rank environment and exits before
anything touches a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_rank_launch_cmd():
    import bench
    argv = ["--gpus", "4", "--steps", "7"]
    args = bench.parse(argv)
    cmd = bench.rank_launch_cmd(args, argv, 29555, pmc_file="/tmp/x.json")
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29555"
    script = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[script + 1:] == argv + ["--pmc-file", "/tmp/x.json"]
    # no PMC figures: the ranks must not run their own PMC passes
    assert bench.rank_launch_cmd(args, argv, 1)[-1] == "--no-pmc"


def test_gpus2_spawns_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rank-probe", "--steps", "3"],
                       cwd=ROOT, env=_env(GSR_DIST_BACKEND="gloo"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 for d in lines)
    assert sorted(d["local_rank"] for d in lines) == [0, 1]
    # every rank got the launcher's arguments (and no PMC passes of its own)
    assert all(d["argv"][:5] == ["--gpus", "2", "--rank-probe", "--steps", "3"] and "--no-pmc" in d["argv"]
               for d in lines)


@pytest.mark.parametrize("mode", ["strong", "weak"])
def test_gpus2_views_per_mode(mode):
    """Both modes the driver may run at N = 2: strong scaling (the default: config 4's fixed batch of
    8 views, 4 per rank) and weak scaling (--views-per-rank 8: 8 distinct views per rank, 16 per
    step).  The ranks' views are disjoint and cover the step."""
    extra = ["--views-per-rank", "8"] if mode == "weak" else []
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rank-probe"] + extra,
                       cwd=ROOT, env=_env(GSR_DIST_BACKEND="gloo"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = sorted((json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")), key=lambda d: d["rank"])
    assert [d["rank"] for d in lines] == [0, 1] and all(d["scaling"] == mode for d in lines)
    views = [v for d in lines for v in d["views"]]
    assert len(views) == len(set(views)) == lines[0]["views_step"]
    if mode == "weak":
        assert all(len(d["views"]) == 8 for d in lines) and lines[0]["views_step"] == 16
        assert lines[0]["n_ring"] == 16 and sorted(views) == list(range(16))
    else:
        assert all(len(d["views"]) == 4 for d in lines) and sorted(views) == list(range(8))


def test_world_size_mismatch_fails():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--rank-probe"],
                       cwd=ROOT, env=_env(WORLD_SIZE="2", RANK="0"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.skipif(os.environ.get("GSR_DIST_BACKEND", "nccl") != "nccl", reason="default backend overridden")
def test_rccl_needs_enough_gpus():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has the GPUs")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rank-probe"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "needs 2 GPUs" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["strong", "weak"])
def test_gpus2_gloo_rehearsal_on_one_gpu(mode):
    """The driver's `python bench.py --gpus 2` on the one GPU of the test box, both scaling modes, with
    the ranks over gloo (GSR_DIST_BACKEND; the 8-GPU nodes use RCCL): two ranks start from one
    torch.distributed.run child, each renders its views, the gradients are all-reduced, rank 0 prints
    one JSON line with n_gpus 2 and the mode's scaling and views per step (config 4's step at full
    size: 1M Gaussians, 1080p)."""
    extra = ["--views-per-rank", "8"] if mode == "weak" else []
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-aux", "--no-pmc", "--no-single-view"] + extra,
                       cwd=ROOT, env=_env(GSR_DIST_BACKEND="gloo"), capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 2 and d["scaling"] == mode and d["value"] > 0 and d["steps"] == 2
    assert d["config"]["views_per_step"] == (16 if mode == "weak" else 8), d["config"]
