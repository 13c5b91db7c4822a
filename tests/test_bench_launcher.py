"""bench.py's multi-GPU launch paths, without a GPU (CPU suite).

`python bench.py --gpus N` with no WORLD_SIZE in the environment must drive N ranks itself: the
parent starts N child processes, never touching a GPU; rank 0's line carries n_gpus == N and every
rank's step time.  cpu_baseline is an N = 1 figure (the reference pluglets on the host cores, rank 0 of
a one-GPU run), so an N > 1 line carries none.  --dry-run swaps the device work for an empty timed
region on gloo, so the launcher, rendezvous and max-over-ranks reduction run here.  A WORLD_SIZE that disagrees
with --gpus is refused."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
ORACLE = os.path.join(ROOT, "oracle", "liboracle.so")


def _run(args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.skipif(not os.path.exists(ORACLE), reason="oracle not built (make -C oracle)")
@pytest.mark.parametrize("config", ["k16", "k32r8"])
def test_spawn_path_two_ranks(config):
    p = _run(["--gpus", "2", "--config", config, "--dry-run", "--steps", "2", "--warmup", "1",
              "--cpu-blocks", "64", "--cpu-seconds", "0.5"], {"PQUIC_BENCH_SHARE_GPU": "1"})
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 2 and d["dry_run"] is True
    assert len(d["per_rank_ms_per_step"]) == 2
    assert d["cpu_baseline"] is None  # timed at N = 1 only


@pytest.mark.skipif(not os.path.exists(ORACLE), reason="oracle not built (make -C oracle)")
@pytest.mark.parametrize("config", ["k16", "k32r8"])
def test_single_rank_carries_the_cpu_baseline(config):
    p = _run(["--gpus", "1", "--config", config, "--dry-run", "--steps", "2", "--warmup", "1",
              "--cpu-blocks", "64", "--cpu-seconds", "0.5"])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    cpu = d["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] >= 1
    if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libfecref.so")):
        assert cpu["kind"] == "reference"
        assert ("decode" in cpu["sample"]) == (config == "k16")


@pytest.mark.parametrize("share", [False, True])
def test_spawn_path_rank_devices(share):
    """Each child rank drives the GPU of its LOCAL_RANK (cuda:0..N-1); only the rehearsal knob folds
    ranks onto the devices present (none here, so all onto 0)."""
    p = _run(["--gpus", "3", "--dry-run", "--no-cpu", "--steps", "1", "--warmup", "0"],
             {"PQUIC_BENCH_SHARE_GPU": "1"} if share else {"PQUIC_BENCH_SHARE_GPU": "0"})
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 3
    assert d["per_rank_device"] == ([0, 0, 0] if share else [0, 1, 2])


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "4", "--dry-run", "--no-cpu"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr


def test_single_gpu_dry_run_line():
    p = _run(["--gpus", "1", "--dry-run", "--no-cpu"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 1 and d["cpu_baseline"] is None


def test_launcher_never_opens_the_gpu():
    """The launcher counts GPUs in a throw-away child process and checks, before it starts the ranks,
    that it holds no GPU device file (/dev/kfd, /dev/dri/*) itself; without enough GPUs (none here) it
    exits with code 2 and says how many it saw."""
    sys.path.insert(0, ROOT)
    import bench
    before = bench.gpu_device_fds()
    n = bench.visible_gpu_count()
    assert n >= 0
    assert bench.gpu_device_fds() == before == [], "counting GPUs opened a device file in this process"
    if n >= 2:
        pytest.skip("enough GPUs visible for two ranks")
    p = _run(["--gpus", "2", "--no-cpu"], {"PQUIC_BENCH_SHARE_GPU": "0"})
    assert p.returncode == 2, p.stderr[-2000:]
    assert f"--gpus 2 but {n} GPU(s) visible" in p.stderr


def test_gpus_default_follows_world_size():
    """Under a launcher that sets WORLD_SIZE (torchrun --nproc-per-node N bench.py) without --gpus, the
    rank count is WORLD_SIZE; an explicit --gpus that disagrees is refused (above)."""
    p = _run(["--dry-run", "--no-cpu", "--steps", "1", "--warmup", "0"],
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 0, p.stderr[-2000:]
    assert _line(p.stdout)["n_gpus"] == 1
