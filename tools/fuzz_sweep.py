"""GPU-box: a longer seeded randomized parity sweep than tests/test_fuzz_gpu.py (same case
generator and oracle semantics, other seeds), run for a time budget; prints one progress line per
case and a JSON summary of the worst deviations (PESQ / STOI / ESTOI vs the oracle run on each
unpadded row alone, NaN-pattern mismatches, joint-vs-separate bitwise mismatches).

    python tools/fuzz_sweep.py --seconds 240 --first-seed 1000 > gpurun_out/fuzz.json
"""
import argparse
import json
import os
import sys
import time
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from tests.test_fuzz_gpu import PESQ_TOL, STOI_TOL, _case, _oracle_row  # noqa: E402
from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seconds", type=float, default=240.0)
ap.add_argument("--first-seed", type=int, default=1000)
a = ap.parse_args()

worst = {"PESQ": 0.0, "STOI": 0.0, "ESTOI": 0.0}
worst_case = {}
nan_mismatch, joint_mismatch, over_tol = [], [], []
rows = cases = 0
rates = {}
t0 = time.perf_counter()
seed = a.first_seed
while time.perf_counter() - t0 < a.seconds:
    sr, B, L, lens, ragged, scale, pad = _case(seed)
    c, n, _ = speech_like_pairs(B, L, sr, seed=seed, device="cuda")
    c, n = c * scale, n * scale
    if pad:
        cw = torch.zeros(B, L + pad, device="cuda")
        nw = torch.zeros(B, L + pad, device="cuda")
        cw[:, :L], nw[:, :L] = c, n
        c, n = cw[:, :L], nw[:, :L]
    lt = torch.as_tensor(lens, dtype=torch.int32) if ragged else None
    gp = [d["PESQ"] for d in PESQ(sr, use_gpu=True)(c, n, lengths=lt)]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            rs = STOI(sr, use_gpu=True)(c, n, lengths=lt)
        except TypeError:
            rs = [{"STOI": float("nan"), "ESTOI": float("nan")}] * B
        rj = PESQ_STOI(sr, use_gpu=True)(c, n, lengths=lt)
    got = np.array([gp, [d["STOI"] for d in rs], [d["ESTOI"] for d in rs]], dtype=np.float64).T
    cc, nn = c.cpu().numpy(), n.cpu().numpy()
    want = np.array([_oracle_row(cc[b, :lens[b]], nn[b, :lens[b]], sr) for b in range(B)])
    tag = f"seed {seed}: sr {sr} B {B} L {L} ragged {ragged} scale {scale} pad {pad}"
    for i, key in enumerate(("PESQ", "STOI", "ESTOI")):
        g, w = got[:, i], want[:, i]
        if not np.array_equal(np.isnan(g), np.isnan(w)):
            nan_mismatch.append(f"{key} {tag}")
        ok = ~np.isnan(w) & ~np.isnan(g)
        if ok.any():
            d = float(np.max(np.abs(g[ok] - w[ok])))
            if d > worst[key]:
                worst[key], worst_case[key] = d, tag
            if d > (PESQ_TOL if key == "PESQ" else STOI_TOL):
                over_tol.append(f"{key} {d:.2e} {tag}")
        if not np.array_equal(np.array([r[key] for r in rj]), got[:, i], equal_nan=True):
            joint_mismatch.append(f"{key} {tag}")
    rows += B
    cases += 1
    rates[sr] = rates.get(sr, 0) + B
    print(f"case {cases} {tag}: max |d| PESQ {worst['PESQ']:.2e} STOI {worst['STOI']:.2e} "
          f"ESTOI {worst['ESTOI']:.2e}", file=sys.stderr, flush=True)
    seed += 1

print(json.dumps({"cases": cases, "rows": rows, "seeds": [a.first_seed, seed - 1], "rows_per_rate": rates,
                  "max_abs_dev": worst, "worst_case": worst_case, "tolerance": {"PESQ": PESQ_TOL, "STOI": STOI_TOL},
                  "over_tolerance": over_tol, "nan_pattern_mismatch": nan_mismatch,
                  "joint_vs_separate_mismatch": joint_mismatch, "seconds": round(time.perf_counter() - t0, 1)}))
