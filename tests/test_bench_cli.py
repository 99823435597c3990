"""bench.py's multi-GPU contract on the CPU: `--gpus N` is honoured with and
without a launcher.  --rehearse runs the rank plumbing
only (gloo process group, barrier-bracketed timing, max over ranks, rank 0's
single JSON line) -- the GPU path is exercised by the driver's runs."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_without_launcher_spawns_n_ranks(n):
    p = _run(["--gpus", str(n), "--rehearse", "--steps", "4", "--warmup", "0", "--dist-backend", "gloo"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["ranks_timed"] == n and rec["rehearsal"] is True


@pytest.mark.timeout(120)
def test_launcher_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--rehearse"], _env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr


@pytest.mark.timeout(120)
def test_one_gpu_rehearsal_single_rank():
    p = _run(["--rehearse", "--steps", "2"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 1


@pytest.mark.timeout(300)
def test_under_torch_distributed_run():
    """The driver's launcher form: torch.distributed.run with --nproc-per-node N and --gpus N."""
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29613", BENCH, "--gpus", "2", "--rehearse",
                        "--steps", "3"], env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    recs = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(recs) == 1 and recs[0]["n_gpus"] == 2


def test_resolution_override():
    """--resolution keeps the config's world, flags and GI schedule and changes only the frame size
    (odd sizes included); the metric's description names the new size."""
    import importlib
    import sys as _sys
    _sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    from rvgrt_amd.configs import CONFIGS
    c = bench.bench_config("c4", "1707x961")
    base = CONFIGS["c4"]
    assert (c.width, c.height) == (1707, 961)
    assert (c.log2_n, c.flags, c.gi_sweeps, c.gi_per_frame) == (base.log2_n, base.flags, base.gi_sweeps, base.gi_per_frame)
    assert "1707x961" in c.describe and "3840x2160" not in c.describe
    assert bench.bench_config("c3") is CONFIGS["c3"]
    with pytest.raises(SystemExit):
        bench.bench_config("c3", "1x5")


def test_world_override():
    import importlib
    import sys as _sys
    _sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    c = bench.bench_config("c4", world=9)
    assert c.log2_n == 9 and c.n == 512 and "512^3" in c.describe and "1024^3" not in c.describe
    c = bench.bench_config("c4", "1280x720", 11)
    assert (c.width, c.height, c.n) == (1280, 720, 2048)
    with pytest.raises(SystemExit):
        bench.bench_config("c4", world=12)


def test_recorded_bench_line_keeps_the_contract():
    """The bench line the driver parses, as last recorded on the GPU (profiles/r06/final/driver_bench.json):
    every contract key, the roofline object (algorithmic bytes / launch time against the 8 TB/s peak,
    with the PMC traffic) and the CPU baseline object."""
    path = os.path.join(ROOT, "profiles", "r06", "final", "driver_bench.json")
    d = json.loads(open(path).read().strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["vs_baseline"] is None
    assert d["config"]["workload"] == "c4" and "model" not in d["config"]
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    # achieved = algorithmic bytes per launch / the measured launch time
    assert abs(rf["achieved"] - rf["algorithmic_bytes_per_launch"] / (rf["avg_launch_ms"] * 1e-3) / 1e9) < 0.01 * rf["achieved"]
    assert rf["traffic"] and rf["traffic"] > 0
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] == "port" and cb["cores"] >= 1
    # value = rays per frame x frames per second
    assert abs(d["value"] - d["rays_per_frame"] / (d["ms_per_step"] * 1e-3) / 1e6) < 0.01 * d["value"]
