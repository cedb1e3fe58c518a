"""bench.py's contract pieces that need no GPU: the metric is BASELINE.json's, the defaults are the
1-GPU headline configuration, the CPU baseline leg returns the contract's fields on a bounded
sample, and the roofline's counters come from the PMC summary of the timed library build."""
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


def test_pmc_summary_is_chosen_by_build_id_and_size(tmp_path, monkeypatch):
    """The roofline's counters come from the PMC summary recorded on the timed library build at
    the bench's per-launch size (its "_meta"), never from whichever directory sorts last."""
    prof = tmp_path / "profiles"
    for name, bid, rows, hbm in (("r9_zz", "other", 4096, 1), ("r1_a", "abc123", 4096, 7e9),
                                 ("r9_b", "abc123", 2048, 2)):
        (prof / name).mkdir(parents=True)
        d = {"fsem::pesq::pesq_front<true, false, false>": {"hbm_bytes": hbm, "SQ_INSTS_VALU": 1e9,
                                                              "SQ_WAVE_CYCLES": 4e9, "SQ_WAIT_INST_ANY": 1e9},
             "_meta": {"build_id": bid, "rows_per_launch": rows, "length": 160000}}
        (prof / name / "pmc_summary.json").write_text(json.dumps(d))
    monkeypatch.setattr(bench, "HERE", str(tmp_path))
    summ, src = bench.pmc_summary_for("abc123", 4096, 160000)
    assert src == os.path.join("profiles", "r1_a", "pmc_summary.json")
    assert bench.pmc_kernel(summ, bench.FRONT_KERNELS[True])["hbm_bytes"] == 7e9
    summ, src = bench.pmc_summary_for("nope", 4096, 160000)
    assert summ == {} and src.startswith("none")
    assert bench.pmc_summary_for("abc123", 64, 160000)[0] == {}


def test_bound_is_derived_from_the_counters():
    assert bench.derive_bound({}) == "unmeasured"
    assert bench.derive_bound({"hbm": 0.2, "valu": 0.25, "lds": 0.4}) == "latency"
    assert bench.derive_bound({"hbm": 0.8, "valu": 0.25, "lds": 0.4}) == "hbm"
    assert bench.derive_bound({"hbm": 0.3, "valu": 0.7, "lds": 0.65}) == "valu"
    assert bench.derive_bound({"hbm": 0.3, "valu": 0.2, "lds": 0.9, "wait_inst_share": 0.5}) == "lds"


def test_step_roofline():
    r = bench.step_roofline(4096, 160000, 7.0)
    assert r["algorithmic_bytes"] == 4096 * (2 * 160000 * 4 + 12)
    assert abs(r["hbm_frac"] - r["algorithmic_bytes"] / 7e-3 / 8e12) < 1e-4
    assert abs(r["fp32_frac"] - 4096 * 53e6 / 7e-3 / 157.3e12) < 1e-4


def test_committed_summaries_carry_meta():
    """Every committed PMC summary names the launch size it was recorded at."""
    import glob
    for f in glob.glob(os.path.join(REPO, "profiles", "*", "pmc_summary*.json")):
        m = json.load(open(f)).get("_meta")
        assert m is None or {"rows_per_launch", "length"} <= set(m), f


def test_single_process_rejects_other_workloads(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--single-process", "--workload", "c3"])
    import pytest
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 2


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
