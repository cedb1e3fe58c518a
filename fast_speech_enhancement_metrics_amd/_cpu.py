"""CPU mode of the metrics (``use_gpu=False``), the reference's CPU behaviour.

Batched torch/scipy implementation of the same math the HIP engine runs:
  PESQ: fast_se_metrics/PESQ.py:92-245, utils/bark.py:169-204, utils/loudness.py:48-67
  STOI: fast_se_metrics/STOI.py:26-205
The level-alignment band-pass runs as a float64 second-order-section cascade and the
pre-emphasis as a float64 IIR (scipy C loops); spectra via torch.stft.  STOI's
``normalize`` is deterministic here: its 1e-12 * randn term taken in expectation (zero-variance
rows map to 0, rows far below 1e-12 to ~0, as the engine and the oracle).
"""
from __future__ import annotations

import math
import threading

import numpy as np
import torch
from scipy.signal import butter, lfilter, sosfilt, tf2zpk, zpk2sos

from . import _tables as T

# ----------------------------------------------------------------------------- PESQ constants
_NB = 49
_EDGES = np.concatenate([[0], np.cumsum(T.BINS_PER_BAND)])
_FBANK = torch.zeros(_NB, 256, dtype=torch.float64)
for _i in range(_NB):
    _FBANK[_i, _EDGES[_i]:_EDGES[_i + 1]] = 1.0
_CORR = torch.tensor(T.POW_DENS_CORRECTION, dtype=torch.float64) * T.SP_16K
_THR = torch.tensor(T.ABS_THRESH_POWER, dtype=torch.float64)
_EXP = ((6 / (torch.tensor(T.CENTRE_BARK) + 2.0)).clamp(1.0, 2.0) ** 0.15 * T.ZWICKER_POWER).to(torch.float64)
_WB = torch.tensor(T.WIDTH_BARK, dtype=torch.float64)
_TW = float(_WB[1:].sum())
_bb, _ba = butter(5, [325, 3250], fs=16000, btype="band")
_BP_B = np.asarray(_bb, dtype=np.float32).astype(np.float64)
_BP_A = np.asarray(_ba, dtype=np.float32).astype(np.float64)
_z, _p, _k = tf2zpk(_BP_B, _BP_A)
# numerator is exactly g * (1 - z^-2)^5: place the zeros exactly at +-1
_z = np.array([1.0] * 5 + [-1.0] * 5)
_BP_SOS = zpk2sos(_z, _p, _BP_B[0])
_PRE_B = np.asarray(T.PRE_B, dtype=np.float32).astype(np.float64)
_PRE_A = np.asarray(T.PRE_A, dtype=np.float32).astype(np.float64)
_TAPER = torch.arange(1, 16, dtype=torch.float64) / 16.0


def pesq_frames(L: int) -> int:
    Lp = L + (L % 256)
    return 0 if Lp < 512 else 1 + (Lp - 512) // 256


def bandpass_power(x: np.ndarray) -> np.ndarray:
    """[N, L] -> [N] sum of the squared band-pass output (PESQ.py:94-97, before / (L+5120) / 1.04684)."""
    y = sosfilt(_BP_SOS, x, axis=1)
    return (y * y).sum(axis=1)


def level_scale(power_sum, L: int):
    """1e7 / (power / (L + 5120) / 1.04684): the factor on a row's power (PESQ.py:97-100)."""
    return 1e7 / (power_sum / (L + 5120) / 1.04684)


def pre_emphasize(x: np.ndarray) -> np.ndarray:
    """Edge taper (k/16 on the first and last 15 samples) + the pre-emphasis IIR (PESQ.py:104-113),
    on a copy."""
    x = np.array(x, dtype=np.float64)
    x[:, :15] *= _TAPER.numpy()
    x[:, -15:] *= _TAPER.numpy()[::-1]
    return lfilter(_PRE_B, _PRE_A, x, axis=1)


def power_spectrum(x: torch.Tensor) -> torch.Tensor:
    """[N, L] -> [N, F, 257]: pad by L % 256 (PESQ.py:128-130), Hann-512 / hop-256 |rFFT|^2, the
    DC bin zeroed (PESQ.py:133-136)."""
    pad = x.shape[1] % 256
    if pad:
        x = torch.nn.functional.pad(x, (0, pad))
    spec = torch.stft(x, n_fft=512, hop_length=256, win_length=512,
                      window=torch.hann_window(512, dtype=x.dtype, device=x.device),
                      center=False, return_complex=True).abs().square().transpose(1, 2)
    spec[:, :, 0] = 0.0
    return spec


def bark_bands(spec: torch.Tensor) -> torch.Tensor:
    """[N, F, 257] -> [N, F, 49] (bark.py:203-204)."""
    return torch.einsum("ij,klj->kli", _FBANK.to(spec.device), spec[:, :, :-1]) * _CORR.to(spec.device)


def bark_of_rows(x: torch.Tensor) -> torch.Tensor:
    """PESQ.get_bark_bands on [N, L] rows: level alignment, pre-emphasis, spectrum, Bark bands."""
    L = x.shape[1]
    xd = x.detach().to("cpu", torch.float64).numpy()
    xd = xd * np.sqrt(level_scale(bandpass_power(xd), L))[:, None]
    return bark_bands(power_spectrum(torch.from_numpy(pre_emphasize(xd))))


def equalize(c: torch.Tensor, n: torch.Tensor):
    """PESQ.equalize_bark_bands (PESQ.py:142-166) -> (equalised clean, equalised noisy)."""
    thr = _THR.to(c.device)
    silent = (c * (c > thr * 100.0)).sum(2) < 1e7
    keep = (~silent).unsqueeze(-1)
    mc = (c * ((c > thr * 100.0) & keep)).mean(1)
    mn = (n * ((n > thr * 100.0) & keep)).mean(1)
    ratio = ((mn + 1000.0) / (mc + 1000.0)).clamp(0.01, 100.0)
    ec = ratio.unsqueeze(1) * c
    fr = ((ec * (ec > thr)).sum(2) + 5e3) / ((n * (n > thr)).sum(2) + 5e3)
    fr2 = fr.clone()
    fr2[:, 1:] = 0.8 * fr[:, 1:] + 0.2 * fr[:, :-1]
    return ec, fr2.clamp(3e-4, 5.0).unsqueeze(-1) * n


def loudness(p: torch.Tensor) -> torch.Tensor:
    thr, ex = _THR.to(p.device), _EXP.to(p.device)
    v = (2.0 * thr) ** ex * ((0.5 + 0.5 * p / thr) ** ex - 1.0)
    return torch.where(p <= thr, torch.zeros_like(v), v) * T.SL_16K


def frame_disturbances(ec: torch.Tensor, en: torch.Tensor):
    """Per-frame symmetric / asymmetric disturbances after the frame weighting and the clamp at 45
    (PESQ.py:193-224) -> ([B, F], [B, F])."""
    wb = _WB.to(ec.device)
    lc, ln = loudness(ec), loudness(en)
    d = ln - lc
    d = d.sign() * (d.abs() - 0.25 * torch.minimum(lc, ln)).clamp(min=0)
    sym = (math.sqrt(_TW) * torch.sqrt(((wb * d)[:, :, 1:] ** 2).sum(2))).clamp(min=1e-20)
    a = ((en + 50.0) / (ec + 50.0)) ** 1.2
    a = torch.where(a < 3.0, torch.zeros_like(a), a).clamp(max=12.0)
    asym = (wb * d * a)[:, :, 1:].abs().sum(2).clamp(min=1e-20)
    thr = _THR.to(ec.device)
    w = (((ec * (ec > thr)).sum(2) + 1e5) / 1e7) ** 0.04
    return (sym / w).clamp(max=45.0), (asym / w).clamp(max=45.0)


def overlapping_sums(v: torch.Tensor) -> torch.Tensor:
    """[B, F] -> [B]: L6 within 20-frame windows (hop 10), L2 across windows (PESQ.py:168-172)."""
    fr_ = v.unfold(1, 20, 10)
    return (fr_ ** 6).mean(2).pow(1.0 / 6.0).square().mean(1).sqrt()


def mos_of(sd: torch.Tensor, ad: torch.Tensor) -> torch.Tensor:
    """PESQ.py:240-243."""
    m = 4.5 - 0.1 * sd - 0.0309 * ad
    return 0.999 + 4.0 / (1.0 + torch.exp(-1.3669 * m + 3.8224))


def pesq_distances(clean: torch.Tensor, noisy: torch.Tensor):
    """PESQ.get_disturbances: [B, L] 16 kHz -> (symmetric, asymmetric) distances [B] float64."""
    B, L = clean.shape
    F = pesq_frames(L)
    if F < 20:
        raise RuntimeError(f"maximum size for tensor at dimension 1 is {max(F, 0)} but size is 20")
    bark = bark_of_rows(torch.cat([clean, noisy], 0))
    ec, en = equalize(bark[:B], bark[B:])
    sym, asym = frame_disturbances(ec, en)
    return overlapping_sums(sym), overlapping_sums(asym)


def pesq(clean: torch.Tensor, noisy: torch.Tensor) -> torch.Tensor:
    """[B, L] 16 kHz float32 -> MOS [B] float64."""
    return mos_of(*pesq_distances(clean, noisy))


# ----------------------------------------------------------------------------- STOI
_SW = torch.hann_window(257)[1:].to(torch.float64)


def _obm() -> torch.Tensor:
    freqs = torch.linspace(0, 5000, 257, dtype=torch.float64)
    k = torch.arange(15, dtype=torch.float64)
    lo = 150 * torch.pow(2.0, (2 * k - 1) / 6)
    hi = 150 * torch.pow(2.0, (2 * k + 1) / 6)
    m = torch.zeros(15, 257, dtype=torch.float64)
    for i in range(15):
        m[i, int(torch.argmin((freqs - lo[i]).abs())):int(torch.argmin((freqs - hi[i]).abs()))] = 1
    return m


_OBM = _obm()
_CLIP = 1 + 10 ** (15 / 20)


def _norm(v: torch.Tensor, dim: int) -> torch.Tensor:
    """STOI.py:113-119 in expectation over its 1e-12 * randn term: the squared norm gains
    N * 1e-24 (N = the normalised dimension's size), the noise averages out of the products."""
    v = v - v.mean(dim=dim, keepdim=True)
    return v / torch.sqrt(v.square().sum(dim=dim, keepdim=True) + v.shape[dim] * 1e-24)


def _estoi_norm(seg: torch.Tensor) -> torch.Tensor:
    """Time, then band normalisation of [S, 15, 30] segments (STOI.py:178-181) in expectation over
    both noise terms: the band normalisation's norm also takes the noise the time normalisation
    left in each element (variance 1e-24 / its row's squared norm, x 14/15 after centring)."""
    c = seg - seg.mean(dim=2, keepdim=True)
    n2 = c.square().sum(dim=2, keepdim=True) + 30e-24
    a = c / n2.sqrt()
    a = a - a.mean(dim=1, keepdim=True)
    q = a.square().sum(dim=1, keepdim=True) + (14 / 15) * (1e-24 / n2).sum(dim=1, keepdim=True) + 15e-24
    return a / q.sqrt()


def stoi(clean: torch.Tensor, noisy: torch.Tensor):
    """[B, L10] 10 kHz -> (stoi [B], estoi [B]) float64; NaN where no 30-frame segment exists."""
    B = clean.shape[0]
    out_s = torch.full((B,), float("nan"), dtype=torch.float64)
    out_e = torch.full((B,), float("nan"), dtype=torch.float64)
    x = clean.to(torch.float64)
    y = noisy.to(torch.float64)
    if x.shape[1] < 256:
        raise RuntimeError("STOI input shorter than one 256-sample frame at 10 kHz")
    xf = x.unfold(1, 256, 128) * _SW
    yf = y.unfold(1, 256, 128) * _SW
    e = 20 * torch.log10(xf.norm(dim=2) + 1e-9)
    keep = (e.amax(1, keepdim=True) - 40 - e) < 0
    win512 = torch.zeros(512, dtype=torch.float64)
    win512[128:384] = _SW
    for b in range(B):
        kx, ky = xf[b][keep[b]], yf[b][keep[b]]
        n = kx.shape[0]
        nseg = n - 31
        if nseg <= 0:
            continue
        length = (n + 1) * 128
        ox = torch.zeros(length, dtype=torch.float64)
        oy = torch.zeros(length, dtype=torch.float64)
        idx = (128 * torch.arange(n)[:, None] + torch.arange(256)[None, :]).reshape(-1)
        ox.index_add_(0, idx, kx.reshape(-1))
        oy.index_add_(0, idx, ky.reshape(-1))
        sp = torch.stft(torch.stack([ox, oy]), n_fft=512, hop_length=128, win_length=512, window=win512,
                        center=False, return_complex=True).abs().square()            # [2, 257, T]
        tob = torch.sqrt(torch.matmul(_OBM, sp))                                      # [2, 15, T]
        segs = tob.unfold(2, 30, 1)[:, :, :nseg]                                      # [2, 15, S, 30]
        cx, cy = segs[0].transpose(0, 1), segs[1].transpose(0, 1)                     # [S, 15, 30]
        alpha = cx.norm(dim=2, keepdim=True) / (cy.norm(dim=2, keepdim=True) + 1e-9)
        yc = torch.minimum(cy * alpha, cx * _CLIP)
        out_s[b] = (_norm(cx, 2) * _norm(yc, 2)).sum() / 15 / nseg
        out_e[b] = (_estoi_norm(cx) * _estoi_norm(cy)).sum() / 30 / nseg
    return out_s, out_e


# torch's intra-op thread count is process-wide: concurrent _host_map calls (metric calls from
# several Python threads) share one save / restore, counted under a lock -- the first call in
# saves the caller's setting and sets 1, the last call out restores it.
_threads_lock = threading.Lock()
_threads_depth = 0
_threads_saved = 1


def _threads_enter() -> int:
    """Pool size for a row map (the caller's thread count); torch's intra-op threads -> 1."""
    global _threads_depth, _threads_saved
    with _threads_lock:
        if _threads_depth == 0:
            _threads_saved = torch.get_num_threads()
            torch.set_num_threads(1)
        _threads_depth += 1
        return _threads_saved


def _threads_exit() -> None:
    global _threads_depth
    with _threads_lock:
        _threads_depth -= 1
        if _threads_depth == 0:
            torch.set_num_threads(_threads_saved)


def host_threads() -> int:
    """torch's intra-op thread count as the caller set it (not the 1 of a row map in flight)."""
    with _threads_lock:
        return _threads_saved if _threads_depth > 0 else torch.get_num_threads()


def _host_map(fn, items):
    """[fn(item) for item in items] on up to host_threads() host threads, torch's own intra-op
    parallelism set to 1 meanwhile (rows are independent; scipy's filters and torch's kernels
    release the GIL, so row chunks run concurrently: 2.5x for PESQ and 1.4x for STOI on 8 cores
    against one call with 8 intra-op threads)."""
    items = list(items)
    if min(host_threads(), len(items)) <= 1:
        return [fn(it) for it in items]
    from concurrent.futures import ThreadPoolExecutor
    nt = min(_threads_enter(), len(items))
    try:
        with ThreadPoolExecutor(max(nt, 1)) as ex:
            return list(ex.map(fn, items))
    finally:
        _threads_exit()


def _cat(outs):
    if isinstance(outs[0], tuple):
        return tuple(torch.cat([o[i] for o in outs]) for i in range(len(outs[0])))
    return torch.cat(outs)


def rows_parallel(fn, clean: torch.Tensor, noisy: torch.Tensor):
    """fn(clean, noisy) -> [B] tensor(s), computed over contiguous row chunks on the host's
    threads (one chunk per thread) and concatenated in row order."""
    B = clean.shape[0]
    nt = max(1, min(host_threads(), B))
    bounds = [(i * B // nt, (i + 1) * B // nt) for i in range(nt)]
    return _cat(_host_map(lambda lh: fn(clean[lh[0]:lh[1]], noisy[lh[0]:lh[1]]), bounds))


def per_row(fn, clean: torch.Tensor, noisy: torch.Tensor, lengths: torch.Tensor):
    """Variable-length CPU mode: ``fn`` on each unpadded row alone (batching.py); rows ``fn``
    rejects as too short score NaN.  Returns what ``fn`` returns, stacked over rows."""
    def one(b):
        n = int(lengths[b])
        try:
            return fn(clean[b:b + 1, :n], noisy[b:b + 1, :n])
        except RuntimeError:
            return None

    outs = _host_map(one, range(clean.shape[0]))
    proto = next((o for o in outs if o is not None), None)
    if proto is None:
        proto = torch.zeros(1, dtype=torch.float64) if fn is pesq else (torch.zeros(1, dtype=torch.float64),) * 2
    nan = float("nan")
    if isinstance(proto, tuple):
        return tuple(torch.cat([o[i] if o is not None else torch.full((1,), nan, dtype=torch.float64) for o in outs])
                     for i in range(len(proto)))
    return torch.cat([o if o is not None else torch.full((1,), nan, dtype=torch.float64) for o in outs])


# ----------------------------------------------------------------------------- time alignment
# The opt-in P.862-style delay estimation (not in the reference, PESQ.py:19-22; engine:
# csrc/align.hip, which documents the stages), float64 with FFT cross-correlations.
_TA_FRAME, _TA_FINE, _TA_ITERS = 64, 383, 12


def _ta_envelope(x: np.ndarray) -> np.ndarray:
    nfr = x.shape[0] // _TA_FRAME
    e = np.square(x[:nfr * _TA_FRAME].reshape(nfr, _TA_FRAME)).sum(axis=1)
    if nfr == 0:
        return e
    thr = e.mean()
    for _ in range(_TA_ITERS):
        sel = e <= thr
        if not sel.any():
            break
        mu = e[sel].mean()
        thr = 1.001 * (mu + 2.0 * math.sqrt(np.square(e[sel] - mu).mean()))
    return np.where(e > thr, np.log(np.maximum(e, 1e-300) / max(thr, 1e-300)), 0.0)


def _xcorr_window(a: np.ndarray, b: np.ndarray, lo: int, hi: int) -> np.ndarray:
    """c[j - lo] = sum_k a[k] b[k + j] for lags lo <= j <= hi (zero outside the arrays)."""
    from scipy.signal import correlate
    n = a.shape[0]
    full = correlate(b, a, mode="full", method="fft")  # full[j + n - 1] = sum_k a[k] b[k + j]
    out = np.zeros(hi - lo + 1)
    j = np.arange(lo, hi + 1)
    ok = (j > -n) & (j < b.shape[0])
    out[ok] = full[j[ok] + n - 1]
    return out


def _first_max(c: np.ndarray) -> int:
    """Index of the first maximum above zero, or -1."""
    i = int(np.argmax(c)) if c.size else 0
    return i if c.size and c[i] > 0 else -1


def time_align_row(ref: np.ndarray, deg: np.ndarray, max_delay: int) -> int:
    r = np.asarray(ref, dtype=np.float64)
    d = np.asarray(deg, dtype=np.float64)
    er, ed = _ta_envelope(r), _ta_envelope(d)
    nfr = er.shape[0]
    M = min(-(-max_delay // _TA_FRAME), nfr - 1)
    jc = 0
    if M >= 0 and nfr > 0:
        i = _first_max(_xcorr_window(er, ed, -M, M))
        jc = i - M if i >= 0 else 0
    d0 = _TA_FRAME * jc
    L = r.shape[0]
    wr = np.zeros(L)
    wd = np.zeros(L)
    wr[1:] = np.diff(r)
    wd[1:] = np.diff(d)
    i = _first_max(_xcorr_window(wr, wd, d0 - _TA_FINE, d0 + _TA_FINE))
    return d0 - _TA_FINE + i if i >= 0 else d0


# utterance mode (csrc/align.hip stages 5-9; P.862 sections 10.3-10.5)
_TA_MINSPEECH, _TA_JOIN, _TA_MINUTT, _TA_SEARCH, _TA_MAXU, _TA_CHUNK = 4, 50, 50, 75, 16, 5120
_TA_SPLIT_GAIN, _TA_SPLIT_MIN = 1.2, 16


def _ta_utterances(env: np.ndarray) -> list:
    """[(start, end)] frames: speech runs from MINSPEECH frames, joined across gaps < JOIN, kept
    from MINUTT, at most MAXU."""
    act = np.flatnonzero(env > 0)
    utt = []
    if act.size:
        cut = np.flatnonzero(np.diff(act) > 1)
        rs = np.concatenate([[act[0]], act[cut + 1]])
        re = np.concatenate([act[cut] + 1, [act[-1] + 1]])
        keep = re - rs >= _TA_MINSPEECH
        rs, re = rs[keep], re[keep]
        if rs.size:
            cut = np.flatnonzero(rs[1:] - re[:-1] >= _TA_JOIN)  # a gap of JOIN or more starts a new run
            starts = np.concatenate([[rs[0]], rs[cut + 1]])
            ends = np.concatenate([re[cut], [re[-1]]])
            utt = [(int(a), int(b)) for a, b in zip(starts, ends) if b - a >= _TA_MINUTT]
    if len(utt) > _TA_MAXU:
        utt = utt[:_TA_MAXU - 1] + [(utt[_TA_MAXU - 1][0], utt[-1][1])]
    return utt


def _ta_piece_xcorr(wr, wd, a: int, b: int, lo: int, hi: int) -> np.ndarray:
    """c[D - lo] = sum over n in [a, b) of wr[n] wd[n + D], lo <= D <= hi (wd zero outside)."""
    L = wd.shape[0]
    win = np.zeros(b - a + hi - lo)
    s0 = a + lo
    i0, i1 = max(s0, 0), min(s0 + win.shape[0], L)
    if i1 > i0:
        win[i0 - s0:i1 - s0] = wd[i0:i1]
    return _xcorr_window(wr[a:b], win, 0, hi - lo) if b > a else np.zeros(hi - lo + 1)


# P.862 mode (csrc/align.hip stages 10-12; P.862 sections 10.5-10.6 on the fine stage's pieces)
_TA_HIST_T, _TA_HIST_POW, _TA_REL_MIN, _TA_MAXDEPTH, _TA_MAXSEG = 8, 0.125, 0.05, 2, 32


def _ta_hist(pv: np.ndarray, pl: np.ndarray, a: int, b: int, d0: int):
    """(delay, confidence, voting pieces) of pieces [a, b): the first maximum of the triangle-
    smoothed histogram of the voting pieces' peak lags, weighted by peak^0.125."""
    sel = np.flatnonzero(pl[a:b] >= 0) + a
    if sel.size == 0:
        return d0, 0.0, 0
    H = np.zeros(2 * _TA_FINE + 1)
    for i in sel:  # piece order, as the engine adds them
        H[pl[i]] += pv[i] ** _TA_HIST_POW
    k = np.arange(-_TA_HIST_T, _TA_HIST_T + 1)
    S = np.convolve(H, (_TA_HIST_T + 1 - np.abs(k)).astype(np.float64), mode="same")
    j = int(np.argmax(S))
    return d0 - _TA_FINE + j, float(S[j] / ((_TA_HIST_T + 1) * H.sum())), int(sel.size)


def _ta_split_p862(pv, pl, a: int, b: int, d0: int, depth: int) -> list:
    """[(piece offset from a, delay)]: pieces [a, b) split where both halves (two or more voting
    pieces each) disagree by SPLIT_MIN and are more confident than the whole, recursively."""
    D, c, _ = _ta_hist(pv, pl, a, b, d0)
    if depth < _TA_MAXDEPTH and b - a >= 4:
        best = None
        for sp in range(a + 2, b - 1):
            dL, cL, nL = _ta_hist(pv, pl, a, sp, d0)
            dR, cR, nR = _ta_hist(pv, pl, sp, b, d0)
            ok = nL >= 2 and nR >= 2 and abs(dL - dR) >= _TA_SPLIT_MIN and cL > c and cR > c
            if ok and (best is None or cL + cR > best[0]):
                best = (cL + cR, sp)
        if best is not None:
            sp = best[1]
            right = _ta_split_p862(pv, pl, sp, b, d0, depth + 1)
            return _ta_split_p862(pv, pl, a, sp, d0, depth + 1) + [(sp - a + o, d) for o, d in right]
    return [(0, D)]


def time_align_utt_row(ref: np.ndarray, deg: np.ndarray, max_delay: int, mode: str = "utterance"):
    """(seg_start [n+1], seg_delay [n], row delay) of one row (csrc/align.hip, utterance or P.862
    mode)."""
    r = np.asarray(ref, dtype=np.float64)
    d = np.asarray(deg, dtype=np.float64)
    L = r.shape[0]
    er, ed = _ta_envelope(r), _ta_envelope(d)
    nfr = er.shape[0]
    M = min(-(-max_delay // _TA_FRAME), nfr - 1) if nfr >= 2 else 0
    jrow = 0
    if nfr >= 2:
        i = _first_max(_xcorr_window(er, ed, -M, M))
        jrow = i - M if i >= 0 else 0
    utt = _ta_utterances(er)
    R = [0] + [_TA_FRAME * ((utt[u - 1][1] + utt[u][0]) // 2) for u in range(1, len(utt))] + [L]
    wins = utt if utt else [(0, nfr)]
    wr = np.zeros(L)
    wd = np.zeros(L)
    wr[1:] = np.diff(r)
    wd[1:] = np.diff(d)
    starts, delays = [], []
    for u, (s, e) in enumerate(wins):
        k0, k1 = max(0, s - _TA_SEARCH), min(nfr, e + _TA_SEARCH)
        jlo, jhi = max(-M, jrow - _TA_SEARCH), min(M, jrow + _TA_SEARCH)
        best, arg = 0.0, None
        for j in range(jlo, jhi + 1):
            ks, ke = max(k0, -j), min(k1, nfr - j)
            c = float(np.dot(er[ks:ke], ed[ks + j:ke + j])) if ke > ks else 0.0
            if c > best:
                best, arg = c, j
        d0 = _TA_FRAME * (arg if arg is not None else jrow)
        m = max(1, -(-(R[u + 1] - R[u]) // _TA_CHUNK))
        P = np.stack([_ta_piece_xcorr(wr, wd, R[u] + i * _TA_CHUNK, min(R[u] + (i + 1) * _TA_CHUNK, R[u + 1]),
                                      d0 - _TA_FINE, d0 + _TA_FINE) for i in range(m)])
        if mode == "p862":
            pl = np.array([_first_max(P[i]) for i in range(m)])
            pv = np.array([P[i, j] if j >= 0 else 0.0 for i, j in enumerate(pl)])
            pl[pv < _TA_REL_MIN * pv.max()] = -1
            for off, D in _ta_split_p862(pv, pl, 0, m, d0, 0):
                if not (delays and delays[-1] == D) and len(delays) < _TA_MAXSEG:
                    starts.append(R[u] + off * _TA_CHUNK)
                    delays.append(D)
            continue
        W = P.sum(axis=0)
        iW = _first_max(W)
        segs = [(0, d0 - _TA_FINE + iW if iW >= 0 else d0)]
        if m >= 4:
            left = np.cumsum(P, axis=0)
            cand = []
            for sp in range(2, m - 1):
                lf, rt = left[sp - 1], W - left[sp - 1]
                iL, iR = _first_max(lf), _first_max(rt)
                vL, vR = (lf[iL] if iL >= 0 else 0.0), (rt[iR] if iR >= 0 else 0.0)
                cand.append((vL + vR, sp, vL, iL, vR, iR))
            tot, sp, vL, iL, vR, iR = max(cand, key=lambda t: t[0])  # first maximum
            vW = W[iW] if iW >= 0 else 0.0
            if vL > 0 and vR > 0 and tot > _TA_SPLIT_GAIN * vW and abs(iL - iR) >= _TA_SPLIT_MIN:
                segs = [(0, d0 - _TA_FINE + iL), (sp * _TA_CHUNK, d0 - _TA_FINE + iR)]
        for off, D in segs:
            if not (delays and delays[-1] == D):
                starts.append(R[u] + off)
                delays.append(D)
    starts.append(L)
    lens = np.diff(starts)
    return np.array(starts), np.array(delays), int(delays[int(np.argmax(lens))])


def time_align_utterances(clean: torch.Tensor, noisy: torch.Tensor, lengths=None, max_delay: int = 16000,
                          mode: str = "utterance"):
    """(aligned [B, L] f32, delays [B], n_seg [B], seg_start [B, 33], seg_delay [B, 32]) int32."""
    c = clean.detach().cpu().numpy()
    n = noisy.detach().cpu().numpy()
    B, L = c.shape
    S = 2 * _TA_MAXU
    out = np.zeros((B, L), dtype=np.float32)
    ds = np.zeros(B, dtype=np.int32)
    ns = np.zeros(B, dtype=np.int32)
    st = np.zeros((B, S + 1), dtype=np.int32)
    sd = np.zeros((B, S), dtype=np.int32)
    rows = [L if lengths is None else int(min(max(int(lengths[b]), 0), L)) for b in range(B)]
    res = _host_map(lambda b: time_align_utt_row(c[b, :rows[b]], n[b, :rows[b]], max_delay, mode), range(B))
    for b, (starts, delays, D) in enumerate(res):
        k = len(delays)
        ns[b], ds[b] = k, D
        st[b, :k + 1] = starts
        sd[b, :k] = delays
        for i in range(k):
            a, e, Dk = int(starts[i]), int(starts[i + 1]), int(delays[i])
            lo, hi = max(a, -Dk), min(e, rows[b] - Dk)
            if hi > lo:
                out[b, lo:hi] = n[b, lo + Dk:hi + Dk]
    return tuple(torch.from_numpy(x) for x in (out, ds, ns, st, sd))


def time_align(clean: torch.Tensor, noisy: torch.Tensor, lengths=None, max_delay: int = 16000):
    """(aligned noisy [B, L] float32, delays [B] int32) of 16 kHz rows (rows past lengths[b] 0)."""
    c = clean.detach().cpu().numpy()
    n = noisy.detach().cpu().numpy()
    B, L = c.shape
    out = np.zeros((B, L), dtype=np.float32)
    ds = np.zeros(B, dtype=np.int32)
    rows = [L if lengths is None else int(min(max(int(lengths[b]), 0), L)) for b in range(B)]
    ds[:] = _host_map(lambda b: time_align_row(c[b, :rows[b]], n[b, :rows[b]], max_delay), range(B))
    for b in range(B):
        m, D = rows[b], int(ds[b])
        lo, hi = max(0, -D), min(m, m - D)
        if hi > lo:
            out[b, lo:hi] = n[b, lo + D:hi + D]
    return torch.from_numpy(out), torch.from_numpy(ds)


# bad intervals (csrc/align.hip ta_bad_*; P.862 section 10.7): the P.862 mode's realignment of
# runs of badly scored frames, then the pooling over the better-scored frames
_BAD_THR, _BAD_GAP, _BAD_MIN, _BAD_MAX, _HOP = 30.0, 4, 5, 16, 256


def bad_runs(sym: np.ndarray) -> list:
    """[(f0, f1)]: runs of frames above BAD_THR, joined across gaps < BAD_GAP, from BAD_MIN
    frames, at most BAD_MAX in order."""
    bad = np.flatnonzero(np.asarray(sym) > _BAD_THR)
    if bad.size == 0:
        return []
    cut = np.flatnonzero(np.diff(bad) > 1)
    rs = np.concatenate([[bad[0]], bad[cut + 1]])
    re = np.concatenate([bad[cut] + 1, [bad[-1] + 1]])
    j = np.flatnonzero(rs[1:] - re[:-1] >= _BAD_GAP)
    s = np.concatenate([[rs[0]], rs[j + 1]])
    e = np.concatenate([re[j], [re[-1]]])
    return [(int(a), int(b)) for a, b in zip(s, e) if b - a >= _BAD_MIN][:_BAD_MAX]


def pesq_frame_scores(clean: torch.Tensor, noisy: torch.Tensor):
    """Per-frame (symmetric, asymmetric) disturbances [B, F] of [B, L] 16 kHz rows."""
    B = clean.shape[0]
    bark = bark_of_rows(torch.cat([clean, noisy], 0))
    ec, en = equalize(bark[:B], bark[B:])
    return frame_disturbances(ec, en)


def realign_bad_row(ref: np.ndarray, deg: np.ndarray, aligned: np.ndarray, starts, delays, sym: np.ndarray):
    """([(f0, f1, delay)], second degraded row) of one unpadded row."""
    L = deg.shape[0]
    out = np.array(aligned, dtype=np.float32, copy=True)
    runs = bad_runs(sym)
    if not runs:
        return [], out
    wr = np.zeros(L)
    wd = np.zeros(L)
    wr[1:] = np.diff(np.asarray(ref, dtype=np.float64))
    wd[1:] = np.diff(np.asarray(deg, dtype=np.float64))
    res = []
    for f0, f1 in runs:
        a, e = _HOP * f0, min(_HOP * f1 + _HOP, L)
        k = int(np.searchsorted(starts, a, side="right")) - 1
        d0 = int(delays[min(max(k, 0), len(delays) - 1)])
        i = _first_max(_ta_piece_xcorr(wr, wd, a, e, d0 - _TA_FINE, d0 + _TA_FINE))
        D = d0 - _TA_FINE + i if i >= 0 else d0
        res.append((f0, f1, D))
        lo, hi = max(a, -D), min(e, L - D)
        out[a:e] = 0.0
        if hi > lo:
            out[lo:hi] = deg[lo + D:hi + D]
    return res, out


def pesq_p862_row(ref: np.ndarray, deg: np.ndarray, aligned: np.ndarray, starts, delays):
    """(MOS, [(f0, f1, delay)]) of one unpadded row already aligned by the P.862 mode."""
    L = ref.shape[0]
    if pesq_frames(L) < 20:
        return float("nan"), []
    c = torch.from_numpy(np.ascontiguousarray(ref, dtype=np.float32)).unsqueeze(0)
    s1, a1 = pesq_frame_scores(c, torch.from_numpy(np.ascontiguousarray(aligned, dtype=np.float32)).unsqueeze(0))
    res, second = realign_bad_row(ref, deg, aligned, starts, delays, s1[0].numpy())
    if res:
        s2, a2 = pesq_frame_scores(c, torch.from_numpy(second).unsqueeze(0))
        s1, a1 = s1.clone(), a1.clone()
        for f0, f1, _ in res:
            if float(s2[0, f0:f1].sum()) < float(s1[0, f0:f1].sum()):
                s1[0, f0:f1] = s2[0, f0:f1]
                a1[0, f0:f1] = a2[0, f0:f1]
    return float(mos_of(overlapping_sums(s1), overlapping_sums(a1))[0]), res


def pesq_p862(clean: torch.Tensor, noisy: torch.Tensor, lengths=None, max_delay: int = 16000):
    """(MOS [B] float64, delays [B] int32, n_bad [B] int32, bad [B, 16, 3] int32) of 16 kHz rows:
    the P.862-mode alignment, then the bad-interval realignment."""
    aligned, ds, ns, st, sd = time_align_utterances(clean, noisy, lengths, max_delay, mode="p862")
    c = clean.detach().cpu().float().numpy()
    n = noisy.detach().cpu().float().numpy()
    a = aligned.numpy()
    B, L = c.shape
    rows = [L if lengths is None else int(min(max(int(lengths[b]), 0), L)) for b in range(B)]

    def one(b):
        k = int(ns[b])
        m = rows[b]
        return pesq_p862_row(c[b, :m], n[b, :m], a[b, :m], st[b, :k + 1].numpy(), sd[b, :k].numpy())

    res = _host_map(one, range(B))
    mos = torch.tensor([r[0] for r in res], dtype=torch.float64)
    nb = torch.zeros(B, dtype=torch.int32)
    bad = torch.zeros(B, _BAD_MAX, 3, dtype=torch.int32)
    for b, (_, iv) in enumerate(res):
        nb[b] = len(iv)
        if iv:
            bad[b, :len(iv)] = torch.tensor(iv, dtype=torch.int32)
    return mos, ds, nb, bad
