"""CPU side of tools/probes/tob_dump.py: the engine's 1/3-octave envelopes against the float64 oracle's
(oracle/stoi_oracle.py, test infrastructure) on the same 10 kHz rows, per band, and the scores
that float64 segment statistics give on each -- which envelope (clean or denoised) moves a row's
STOI away from the exact value.

    python tools/probes/tob_compare.py gpurun_out/TAG/tob_dump.npz [golden_name]   (default tone_probe_10k)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from oracle import stoi_oracle as so  # noqa: E402


def score(tx, ty):
    """STOI of two envelope arrays [15, T] with the oracle's float64 segment math."""
    tx, ty = tx.astype(np.float64), ty.astype(np.float64)
    nseg = tx.shape[1] - 29
    idx = np.arange(nseg)[:, None] + np.arange(30)[None, :]
    xs, ys = tx[:, idx].transpose(1, 0, 2), ty[:, idx].transpose(1, 0, 2)
    alpha = np.sqrt((xs ** 2).sum(2, keepdims=True)) / (np.sqrt((ys ** 2).sum(2, keepdims=True)) + 1e-9)
    yc = np.minimum(ys * alpha, xs * (1 + 10 ** 0.75))
    return (so._normalize(xs, 2) * so._normalize(yc, 2)).sum() / 15 / nseg


def main():
    d = np.load(sys.argv[1])
    name = sys.argv[2] if len(sys.argv) > 2 else "tone_probe_10k"
    tob, kept = d[name + "_tob"], d[name + "_kept"]
    c10, n10 = d[name + "_x10_clean"], d[name + "_x10_noisy"]
    B = c10.shape[0]
    for r in range(B):
        T = int(kept[r]) - 2
        if T < 30:
            continue
        tx_e, ty_e = tob[r][:, :T], tob[B + r][:, :T]
        xs, ys, _, _ = so.remove_silent_frames(c10[r], n10[r])
        tx = so.third_octave_bands(xs.astype(np.float64))
        ty = so.third_octave_bands(ys.astype(np.float64))
        ex = (np.abs(tx_e - tx) / np.abs(tx).mean(1, keepdims=True)).max(1)
        ey = (np.abs(ty_e - ty) / np.abs(ty).mean(1, keepdims=True)).max(1)
        print(f"row {r}: engine STOI {float(d[name + '_stoi'][r]):+.4f} | float64 {score(tx, ty):+.4f} | "
              f"engine clean + float64 denoised {score(tx_e, ty):+.4f} | float64 clean + engine denoised "
              f"{score(tx, ty_e):+.4f}")
        print("   max band error / band mean, clean:   ", " ".join(f"{v:.1e}" for v in ex))
        print("   max band error / band mean, denoised:", " ".join(f"{v:.1e}" for v in ey))


if __name__ == "__main__":
    main()
