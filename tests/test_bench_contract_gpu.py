"""bench.py's one-line JSON contract on a real GPU (the driver parses this line every round): the
required keys and types, the roofline object consistent with itself, the CPU baseline's fields, and the
numbers sane -- on a short run of the default workload and of configs[3]."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _run(args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    return json.loads(lines[0])


def _check_common(d, steps, warmup, scaling="weak"):
    for key, typ in (("metric", str), ("value", (int, float)), ("unit", str), ("n_gpus", int), ("steps", int),
                     ("warmup", int), ("ms_per_step", (int, float)), ("higher_is_better", bool),
                     ("scaling", str), ("dtype", str), ("data", str), ("config", dict), ("roofline", dict)):
        assert isinstance(d.get(key), typ), (key, d.get(key))
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == warmup
    # configs[3] splits a fixed 2^24 blocks over the GPUs (strong); the others fix the work per GPU
    assert d["higher_is_better"] is True and d["scaling"] == scaling and d["dtype"] == "u8"
    assert d["vs_baseline"] is None or isinstance(d["vs_baseline"], (int, float))
    assert d["value"] > 0 and d["ms_per_step"] > 0 and "workload" in d["config"]
    ro = d["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in ro, key
    assert ro["bound"] == "hbm" and ro["unit"] == "GB/s" and ro["peak"] == 8000.0
    assert 0 < ro["achieved"] < ro["peak"]
    assert abs(ro["frac"] - ro["achieved"] / ro["peak"]) < 1e-3
    assert ro["traffic"] is None or ro["traffic"] > 0


@pytest.mark.gpu
def test_bench_line_default_workload():
    d = _run(["--steps", "2", "--warmup", "1", "--no-legs", "--cpu-seconds", "1", "--cpu-blocks", "256"])
    _check_common(d, 2, 1)
    cpu = d["cpu_baseline"]
    assert isinstance(cpu, dict)
    for key in ("value", "unit", "cores", "kind", "sample"):
        assert key in cpu, key
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] in ("reference", "port")
    # the step's algorithmic rate cannot beat the dominant kernel's: value (GiB/s of k*L payload per step)
    # times (k + e) / k bytes per payload byte over two kernels is below the roofline kernel's rate
    assert d["value"] * 2 ** 30 / 1e9 < ro_rate(d)


def ro_rate(d):
    return d["roofline"]["achieved"]


@pytest.mark.gpu
def test_bench_line_k32r8():
    d = _run(["--config", "k32r8", "--steps", "1", "--warmup", "1", "--no-cpu"])
    _check_common(d, 1, 1, scaling="strong")
    assert d["cpu_baseline"] is None
    assert "k32" in d["roofline"]["kernel"] or "<8," in d["roofline"]["kernel"]
    # the line printed only after the byte gate: every pass's sampled repairs decoded back to the sources
    g = d["config"]["encode_gate"]
    assert g["passes_checked"] == d["config"]["passes_per_step"] >= 1
    assert g["blocks_decoded_back"] >= 0.9 * 4096 * g["passes_checked"]
