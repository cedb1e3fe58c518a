"""bench.py's contract pieces that need no GPU: the metric is BASELINE.json's, the defaults are the
1-GPU headline configuration, the CPU baseline leg returns the contract's fields on a bounded
sample, and the roofline's traffic comes from the newest committed PMC summary."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_metric_is_baselines():
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert bench.METRIC == json.load(f)["metric"]


def test_defaults_are_the_headline_config(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.batch, a.length, a.workload) == (1, 4096, 160000, "c2")
    assert a.steps > 0 and a.warmup >= 0 and not a.separate


def test_cpu_oracle_fields():
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(2, 16000, 16000, seed=3)
    out = bench.cpu_oracle(c, n, budget_s=0.0)  # one pair, then the budget stops it
    assert set(out) == {"value", "unit", "cores", "kind", "sample"}
    assert out["kind"] == "port" and out["cores"] == 1 and out["unit"] == "utterances/s"
    assert np.isfinite(out["value"]) and out["value"] > 0
    assert out["sample"].startswith("1 pairs x 16000 samples")
    assert torch.get_num_threads() >= 1


def test_roofline_traffic_from_newest_pmc_summary():
    rounds = sorted(os.listdir(os.path.join(REPO, "profiles")),
                    key=lambda p: [int(t) if t.isdigit() else t for t in __import__("re").split(r"(\d+)", p)])
    newest = [r for r in rounds if os.path.exists(os.path.join(REPO, "profiles", r, "pmc_summary.json"))][-1]
    with open(os.path.join(REPO, "profiles", newest, "pmc_summary.json")) as f:
        rows = json.load(f).get("_meta", {"rows_per_launch": 4096})["rows_per_launch"]
    hbm, src = bench.pmc_traffic(bench.FRONT_KERNELS[True], rows, 160000)
    assert hbm is not None and hbm > 2 * rows * 160000 * 4  # at least the algorithmic input bytes
    assert src == os.path.join("profiles", newest, "pmc_summary.json")
    other = 2048 if rows == 4096 else 4096  # a summary is only used at its own per-launch size
    got = bench.pmc_traffic(bench.FRONT_KERNELS[True], other, 160000)
    assert got == (None, None) or got[1] != src
    assert bench.pmc_traffic(bench.FRONT_KERNELS[True], 64, 160000) == (None, None)  # other sizes: none


def test_cpu_baseline_is_the_use_gpu_false_path():
    """cpu_baseline: the drop-in use_gpu=False call at two batch sizes on the host's cores, median
    after dropping the first 15 % + 1 calls (benchmark_metrics.py:82)."""
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(3, 16000, 16000, seed=4)
    prev = torch.get_num_threads()
    out = bench.cpu_baseline(c, n, batches=(1, 3), calls=3)
    assert torch.get_num_threads() == prev
    assert {"value", "unit", "cores", "kind", "sample", "batches"} <= set(out)
    assert out["kind"] == "port" and out["cores"] == bench.host_cores() and out["value"] > 0
    assert set(out["batches"]) == {"1", "3"} and out["batches"]["3"]["calls"] == 2
    assert out["value"] == out["batches"]["3"]["value"]
    assert "use_gpu=False" in out["sample"] and "threads" in out["sample"]


def test_gpus_above_visible_devices_is_an_error(monkeypatch):
    """--gpus N without a launcher spawns N ranks; more than the visible devices fails loudly."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert bench.spawn_ranks(2) == 2
