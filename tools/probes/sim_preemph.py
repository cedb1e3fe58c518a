"""Float32 simulation of pesq_front's time-parallel pre-emphasis (tiles of 256 chunks x 52 samples,
768-sample warm-up, pass-1 end states, 4-level Hillis-Steele chunk scan, pass 2) in two state
bases -- the transposed direct form (DF2T, round-2 engine) and FIR-then-all-pole (the reference's
lfilter order: w = b * x, then y = w - a1 y[-1] - a2 y[-2]) -- plugged into the oracle's PESQ in
place of its sequential pre-emphasis, on the DC-offset edge golden.  CPU only (study tool).

    python tools/probes/sim_preemph.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from oracle import pesq_oracle as po  # noqa: E402
from tests.conftest import edge_inputs, load_golden  # noqa: E402

CH, PT, WARM, OWN = 52, 256, 768, 12288
TILE = CH * PT
b = np.array([2.740826, -5.4816519, 2.740826], dtype=np.float32).astype(np.float64)
a = np.array([1.0, -1.9444777, 0.94597794], dtype=np.float32).astype(np.float64)
f32 = np.float32


def fma(x, y, z):
    return (np.asarray(x, np.float64) * np.asarray(y, np.float64) + np.asarray(z, np.float64)).astype(f32)


def tables(form):
    """(G [CH, 2], A[d] for d = 1, 2, 4, 8) of the 2-state pre-emphasis in the given basis."""
    if form == "allpoleH":
        form = "allpole"
    if form == "normal":
        # coupled (normal) form of the all-pole part: (u, v) = T (y[n-1], y[n-2]), u = y1 - r c y2,
        # v = r s y2 -- ||M^k|| = r^k
        r = np.sqrt(a[2])
        c = -a[1] / (2 * r)
        sn = np.sqrt(1 - c * c)
        Tm = np.array([[1.0, -r * c], [0.0, r * sn]])
        Gy, Ay = tables("allpole64")
        return (Gy @ Tm.T).astype(f32), [(Tm @ A @ np.linalg.inv(Tm)).astype(f32) for A in Ay], Tm
    if form == "allpole64":
        M = np.array([[-a[1], -a[2]], [1.0, 0.0]])
        K = np.array([1.0, 0.0])
        G = np.zeros((CH, 2))
        P = np.eye(2)
        for k in range(CH - 1, -1, -1):
            G[k] = P @ K
            P = M @ P
        Mch = np.linalg.matrix_power(M, CH)
        return G, [np.linalg.matrix_power(Mch, d) for d in (1, 2, 4, 8)]
    if form == "df2t":
        M = np.array([[-a[1], 1.0], [-a[2], 0.0]])
        K = np.array([b[1] - a[1] * b[0], b[2] - a[2] * b[0]])
    else:  # all-pole states (y[n-1], y[n-2]) driven by w
        M = np.array([[-a[1], -a[2]], [1.0, 0.0]])
        K = np.array([1.0, 0.0])
    G = np.zeros((CH, 2))
    P = np.eye(2)
    for k in range(CH - 1, -1, -1):
        G[k] = P @ K
        P = M @ P
    Mch = np.linalg.matrix_power(M, CH)
    A = [np.linalg.matrix_power(Mch, d).astype(f32) for d in (1, 2, 4, 8)]
    return G.astype(f32), A


def tile_filter(x, form):
    """Pre-emphasis of one tile's samples x [TILE] (zero state at the tile start) -> y [TILE]."""
    tb = tables(form)
    G, A = tb[0], tb[1]
    ch = x.reshape(PT, CH).astype(f32)
    xm1 = np.concatenate([[0.0], ch[:-1, -1]]).astype(f32)  # x[-1], x[-2] of each chunk
    xm2 = np.concatenate([[0.0], ch[:-1, -2]]).astype(f32)
    if form == "df2t":
        inp = ch
    else:
        w = np.empty_like(ch)
        for n in range(CH):
            x1 = ch[:, n - 1] if n >= 1 else xm1
            x2 = ch[:, n - 2] if n >= 2 else (ch[:, n - 1 - 1] if n == 1 and False else (xm1 if n == 1 else xm2))
            w[:, n] = fma(b[0], ch[:, n], fma(b[1], x1, (np.float32(b[2]) * x2).astype(f32)))
        inp = w
    e = np.zeros((PT, 2), f32)
    if form == "allpoleH":
        # end state = sum_n H[n] x[n] + boundary terms of x[-1], x[-2]: H = b0 G[n] + b1 G[n+1] + b2 G[n+2]
        G64 = tables("allpole")[0].astype(np.float64)
        Gp = np.vstack([G64, np.zeros((2, 2))])
        H = (b[0] * Gp[:CH] + b[1] * Gp[1:CH + 1] + b[2] * Gp[2:CH + 2]).astype(f32)
        Hm1 = (b[1] * G64[0] + b[2] * G64[1]).astype(f32)
        Hm2 = (b[2] * G64[0]).astype(f32)
        for i in range(2):
            e[:, i] = fma(Hm2[i], xm2, e[:, i])
            e[:, i] = fma(Hm1[i], xm1, e[:, i])
        for n in range(CH):
            for i in range(2):
                e[:, i] = fma(H[n, i], ch[:, n], e[:, i])
    else:
      for n in range(CH):
        for i in range(2):
            e[:, i] = fma(G[n, i], inp[:, n], e[:, i])
    for lv, d in enumerate((1, 2, 4, 8)):
        q = np.zeros_like(e)
        q[d:] = e[:-d]
        new = e.copy()
        for i in range(2):
            new[:, i] = fma(A[lv][i, 0], q[:, 0], fma(A[lv][i, 1], q[:, 1], e[:, i]))
        e = new
    z = np.zeros_like(e)
    z[1:] = e[:-1]
    if form == "normal":  # back to (y[n-1], y[n-2]) for the direct-form pass 2
        Ti = np.linalg.inv(tb[2]).astype(f32)
        z = np.stack([fma(Ti[0, 0], z[:, 0], (Ti[0, 1] * z[:, 1]).astype(f32)),
                      fma(Ti[1, 0], z[:, 0], (Ti[1, 1] * z[:, 1]).astype(f32))], 1)
    y = np.empty_like(ch)
    if form == "df2t":
        z0, z1 = z[:, 0].copy(), z[:, 1].copy()
        for n in range(CH):
            xn = ch[:, n]
            yn = fma(b[0], xn, z0)
            z0 = fma(b[1], xn, fma(-a[1], yn, z1))
            z1 = fma(b[2], xn, (np.float32(-a[2]) * yn).astype(f32))
            y[:, n] = yn
    else:
        y1, y2 = z[:, 0].copy(), z[:, 1].copy()
        for n in range(CH):
            yn = fma(-a[1], y1, fma(-a[2], y2, inp[:, n]))
            y2, y1 = y1, yn
            y[:, n] = yn
    return y.reshape(-1)


def pre_emphasize_sim(x, form):
    L = x.shape[0]
    xt = x.astype(f32).copy()
    xt[:15] *= po._TAPER
    xt[-15:] *= po._TAPER[::-1]
    out = np.zeros(L, f32)
    nseg = -(-L // OWN)
    for g in range(nseg):
        t0 = g * OWN - WARM
        tile = np.zeros(TILE, f32)
        lo, hi = max(t0, 0), min(t0 + TILE, L)
        tile[lo - t0:hi - t0] = xt[lo:hi]
        y = tile_filter(tile, form)
        o_lo, o_hi = g * OWN, min((g + 1) * OWN, L)
        out[o_lo:o_hi] = y[o_lo - t0:o_hi - t0]
    return out


def pesq_with(clean, noisy, form):
    B = clean.shape[0]
    x = np.concatenate([clean, noisy]).astype(f32)
    power = po.level_power(x)
    s = np.sqrt(np.float32(1e7) / power).astype(np.float64)
    pre = np.stack([pre_emphasize_sim(r, form) for r in x]).astype(np.float64) * s
    pad = x.shape[1] % 256
    if pad:
        pre = np.pad(pre, ((0, 0), (0, pad)))
    spec = po.ta.power_spectrogram(pre.astype(f32), 512, 256, po.ta.hann_periodic(512)).astype(np.float32)
    spec[:, :, 0] = 0.0
    bark = po.bark_from_spectrum(spec.astype(np.float64))
    ec, en = po.equalize_bark_bands(bark[:B], bark[B:])
    ld = po.loudness(np.concatenate([ec, en]))
    lc, ln = ld[:B], ld[B:]
    d = ln - lc
    d = np.sign(d) * np.maximum(np.abs(d) - 0.25 * np.minimum(lc, ln), 0.0)
    sym = np.maximum(po.weighted_norm(d, 2), 1e-20)
    asc = ((en + 50.0) / (ec + 50.0)) ** 1.2
    asc = np.minimum(np.where(asc < 3.0, 0.0, asc), 12.0)
    asym = np.maximum(po.weighted_norm(d * asc, 1), 1e-20)
    w = ((po.audible_frame_power(ec, 1.0) + 1e5) / 1e7) ** 0.04
    return po.mos_from_distances(po.overlapping_sums(np.minimum(sym / w, 45)), po.overlapping_sums(np.minimum(asym / w, 45)))


if __name__ == "__main__":
    g = load_golden("edges_16k")
    for name in ("dc100_clean", "dc100_both", "dc1000_both"):
        c, n = (t.numpy() for t in edge_inputs(g, name))
        ref = g[name + "_pesq"]
        for form in ("df2t", "allpole", "normal"):
            print(f"{name:12s} {form:8s} sim - ref {np.round(pesq_with(c, n, form) - ref, 5)}")
    gb = load_golden("pesq_3s")
    x = gb["clean_f"].astype(f32)
    exact = np.stack([po.ta.lfilter(np.ascontiguousarray(r[None]), po._PRE_A, po._PRE_B)[0] for r in x])
    for form in ("df2t", "allpole", "normal"):
        sim = np.stack([pre_emphasize_sim(np.concatenate([r[:15] / po._TAPER, r[15:-15], r[-15:] / po._TAPER[::-1]]), form)
                        for r in x])
        err = np.abs(sim.astype(np.float64) - exact).max() / np.abs(exact).max()
        print(f"pesq_3s      {form:8s} sim - ref {np.round(pesq_with(gb['clean_f'], gb['noisy_f'], form) - gb['pesq'], 5)}"
              f"  pre-emphasis max rel err vs sequential {err:.2e}")
