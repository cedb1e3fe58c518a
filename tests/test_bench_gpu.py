"""bench.py end to end on the GPU at a small size (the driver's contract: one JSON line on stdout
with the metric, throughput, roofline of the dominant kernel and the CPU legs), run as a child
process like the driver runs it."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def test_bench_json_line_contract():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--batch", "64", "--length", "48000",
                          "--steps", "2", "--warmup", "1", "--kernel-reps", "2", "--cpu-seconds", "0.5",
                          "--cpu-calls", "2"],
                         cwd=REPO, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout  # the result line is the only line on stdout
    d = json.loads(lines[0])
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert d["metric"] == json.load(f)["metric"]
    for key in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "cpu_oracle", "scores_path"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and abs(d["value"] - 64 * 1e3 / d["ms_per_step"]) < 1e-2 * d["value"]
    r = d["roofline"]
    # bound derived from this build's counters: at this size no summary exists -> "unmeasured"
    assert r["bound"] in ("hbm", "valu", "lds", "latency", "unmeasured") and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["library_build_id"] and "step" in r and r["step"]["ms_per_step"] > 0
    assert 0 < r["step"]["hbm_frac"] < 1 and 0 < r["step"]["fp32_frac"] < 1
    assert r["algorithmic_bytes_per_launch"] == 2 * 64 * 48000 * 4
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["traffic"] is None  # PMC traffic is only recorded at the bench configuration
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0 and set(c["batches"]) == {"4", "64"}
    assert d["cpu_oracle"]["cores"] == 1 and d["cpu_oracle"]["value"] > 0
    assert d["scores_path"]["value"] > 0


def test_bench_gpus_beyond_visible_fails():
    """--gpus N without a launcher on a box with fewer devices: a clear error, not a 1-GPU run."""
    import torch
    n = torch.cuda.device_count() + 1
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "1"],
                         cwd=REPO, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "visible" in out.stderr and out.stdout.strip() == ""


def test_bench_rccl_path_one_rank_pipelined():
    """The driver's multi-GPU launch form (torch.distributed.run, RCCL) with one rank, at the
    bench batch (the drop-in call's list plus its [B, 3] scores, all-gathered): one JSON line,
    n_gpus 1."""
    import socket
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for _ in range(3):  # a fresh port when another process took the probed one (nothing ran yet)
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                              "--master-addr", "127.0.0.1", "--master-port", str(port),
                              os.path.join(REPO, "bench.py"), "--gpus", "1", "--batch", "4096", "--length", "16000",
                              "--steps", "2", "--warmup", "1", "--kernel-reps", "1", "--no-cpu-baseline"],
                             cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
        if "EADDRINUSE" not in out.stderr:
            break
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["config"]["batch_per_gpu"] == 4096


def test_bench_single_process_mode():
    """--single-process: one process drives the devices through PESQ_STOI(devices=N) (here N = 1,
    the 1-GPU box): one JSON line with the throughput of the whole batch."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--single-process",
                          "--batch", "64", "--length", "48000", "--steps", "2", "--warmup", "1"],
                         cwd=REPO, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["config"]["global_batch"] == 64 and d["value"] > 0
    assert "devices=N" in d["config"]["workload"]
