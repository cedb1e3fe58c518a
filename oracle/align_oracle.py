"""ORACLE / TEST INFRASTRUCTURE ONLY -- float64 restatement of the engine's opt-in time alignment
(SURVEY.md 8(f)4).  PARITY UNPINNED against ITU-T P.862 / ludlows' pesq: the reference has no
time alignment (``fast_se_metrics/PESQ.py:19-22``: "1. no time alignment") and no P.862
implementation is importable here, so this module restates the published P.862 section 10
structure as the engine implements it, and the tests pin the engine to it on inputs with a
known delay (``tests/test_align_cpu.py``, ``tests/test_align_gpu.py``):

1. Voice-activity envelopes on 4 ms frames (64 samples at 16 kHz, P.862's ``Downsample``):
   frame energies E[k] = sum of x^2 over the frame; a noise threshold re-estimated 12 times from
   the frames at or below it (mean + 2 standard deviations, times 1.001), starting at mean(E);
   envelope env[k] = log(E[k] / thr) above the threshold, else 0 (P.862 ``apply_VAD``).
2. Crude delay: the lag (in frames, |j| <= M) maximising the plain cross-correlation
   sum_k env_ref[k] env_deg[k + j] (P.862 ``crude_align``); 0 if no lag correlates positively.
3. Fine delay: within +-383 samples of the crude one (P.862 searches +-512 around it at
   16 kHz), the sample lag maximising the cross-correlation of the first differences
   w[n] = x[n] - x[n-1] (n >= 1) of the two signals (a pre-whitened whole-signal form of P.862's
   per-utterance ``time_align`` histogram, which this build does not split into utterances); the
   crude delay if no lag correlates positively.  The window: the crude stage's error on the
   synthetic speech-like pairs reaches ~290 samples (4 ms frames of smooth syllabic envelopes);
   narrower windows, or a decimated intermediate stage, lock onto neighbouring pitch-period peaks
   (measured while choosing the design: +-64 recovered 12 / 24 delays, a decimate-by-4 stage
   248 / 256, the full-rate +-383 window 256 / 256).
4. Delay D > 0 means the degraded signal lags the reference: deg[n] ~ ref[n - D].  The aligned
   degraded row is a[n] = deg[n + D] where 0 <= n + D < L, else 0.

Ties: the first maximum in increasing lag order.

Utterance mode (``align_utterances``; engine ``fsem_time_align_utt_f32``), P.862 section 10.3-10.5
restated with the fine stage above:

5. Utterances (P.862 ``id_searchwindows`` / ``id_utterances``): runs of reference frames with a
   positive envelope, runs shorter than MINSPEECH = 4 frames discarded (P.862's MINSPEECHLGTH);
   runs separated by fewer than JOIN = 50 frames (200 ms) are joined, joined runs shorter than
   MINUTT = 50 frames dropped; at most MAXU = 16 (the rest joins the 16th).
   No utterance: the whole row is one.  Regions: utterance u owns samples [R_u, R_u+1) with
   R_0 = 0, R_u = 64 * floor((end_u-1 + start_u) / 2) (the middle of the gap), R_U = L.
6. Per-utterance crude delay (P.862 ``crude_align`` on the utterance's search window): the
   envelope correlation over reference frames [start - SEARCHBUF, end + SEARCHBUF) (75 frames,
   300 ms) at lags within SEARCHBUF frames of the row's crude lag (and |j| <= M); the row's
   crude delay if no lag correlates positively.
7. Per-utterance fine delay: the first-difference correlation of step 3 over the region's
   samples, within +-383 of the utterance's crude delay, accumulated over CHUNK = 5120-sample
   pieces of the region (from R_u).
8. Split (P.862 ``utterance_split``, one level): a region of m >= 4 pieces is tried at every
   piece boundary s in [2, m - 2]; left = sum of pieces < s, right = total - left; the split with
   the largest peak(left) + peak(right) (first such s) is taken when both peaks are positive, it
   beats the whole region's peak by SPLIT_GAIN = 1.2 and the two delays differ by at least
   SPLIT_MIN = 16 samples (1 ms).  Segments: the regions, or their two halves, each with its
   delay, consecutive segments of equal delay merged (at most 32 per row); the row's delay is the
   longest segment's (the first of equals).
9. The aligned degraded row: a[n] = deg[n + D_k] for n in segment k where 0 <= n + D_k < L.
"""
from __future__ import annotations

import numpy as np

FRAME = 64        # samples per envelope frame at 16 kHz (4 ms)
FINE = 383        # fine search half-width in samples (767 lags)
VAD_ITERS = 12


def envelope(x: np.ndarray) -> np.ndarray:
    """VAD log-envelope of one row (step 1)."""
    x = np.asarray(x, dtype=np.float64)
    nfr = x.shape[0] // FRAME
    if nfr == 0:
        return np.zeros(0)
    e = np.square(x[:nfr * FRAME].reshape(nfr, FRAME)).sum(axis=1)
    thr = e.mean()
    for _ in range(VAD_ITERS):
        noise = e[e <= thr]
        if noise.size == 0:
            break
        mu = noise.mean()
        sd = np.sqrt(np.mean(np.square(noise - mu)))
        thr = 1.001 * (mu + 2.0 * sd)
    env = np.zeros(nfr)
    above = e > thr
    env[above] = np.log(e[above] / thr)
    return env


def crude_delay(env_r: np.ndarray, env_d: np.ndarray, max_frames: int) -> int:
    """Step 2: crude delay in frames."""
    nfr = min(env_r.shape[0], env_d.shape[0])
    M = min(max_frames, nfr - 1)
    best, arg = 0.0, 0
    for j in range(-M, M + 1):
        if j >= 0:
            c = float(np.dot(env_r[:nfr - j], env_d[j:nfr]))
        else:
            c = float(np.dot(env_r[-j:nfr], env_d[:nfr + j]))
        if c > best:
            best, arg = c, j
    return arg


def fine_delay(ref: np.ndarray, deg: np.ndarray, d0: int) -> int:
    """Step 3: sample delay within +-FINE of d0 (first differences, n >= 1 on both sides)."""
    r = np.asarray(ref, dtype=np.float64)
    d = np.asarray(deg, dtype=np.float64)
    L = r.shape[0]
    wr = np.zeros(L)
    wd = np.zeros(L)
    wr[1:] = np.diff(r)
    wd[1:] = np.diff(d)
    best, arg = 0.0, d0
    for D in range(d0 - FINE, d0 + FINE + 1):
        lo, hi = max(1, 1 - D), min(L, L - D)
        if hi <= lo:
            continue
        c = float(np.dot(wr[lo:hi], wd[lo + D:hi + D]))
        if c > best:
            best, arg = c, D
    return arg


def delay(ref: np.ndarray, deg: np.ndarray, max_delay: int = 16000) -> int:
    """Delay (samples) of one row pair of equal length at 16 kHz."""
    env_r, env_d = envelope(ref), envelope(deg)
    jc = crude_delay(env_r, env_d, -(-max_delay // FRAME))  # 0 for rows under two frames
    return fine_delay(ref, deg, FRAME * jc)


def shift(deg: np.ndarray, D: int) -> np.ndarray:
    """Step 4: the aligned degraded row."""
    L = deg.shape[0]
    out = np.zeros_like(deg)
    lo, hi = max(0, -D), min(L, L - D)
    if hi > lo:
        out[lo:hi] = deg[lo + D:hi + D]
    return out


def align(ref: np.ndarray, deg: np.ndarray, max_delay: int = 16000, lengths=None):
    """(aligned deg [B, L], delays [B]) for [B, L] rows; rows past lengths[b] stay zero."""
    ref = np.atleast_2d(ref)
    deg = np.atleast_2d(deg)
    B, L = ref.shape
    out = np.zeros_like(deg)
    ds = np.zeros(B, dtype=np.int64)
    for b in range(B):
        n = L if lengths is None else int(min(max(lengths[b], 0), L))
        ds[b] = delay(ref[b, :n], deg[b, :n], max_delay)
        out[b, :n] = shift(deg[b, :n], int(ds[b]))
    return out, ds


# ----------------------------------------------------------------------------- utterance mode
MINSPEECH = 4     # frames: shorter speech runs are discarded (P.862 MINSPEECHLGTH)
JOIN = 50         # frames: gaps shorter than this join two speech runs (P.862 JOINSPEECHLGTH)
MINUTT = 50       # frames: shorter joined runs are not utterances
SEARCHBUF = 75    # frames: the crude search window's margin around an utterance
MAXU = 16         # utterances per row
CHUNK = 5120      # samples per fine-stage piece (split points lie between pieces)
SPLIT_GAIN = 1.2
SPLIT_MIN = 16
MAXSEG = 2 * MAXU


def utterances(env_r: np.ndarray) -> list:
    """Step 5: [(start, end)] frames of the reference's utterances."""
    act = np.asarray(env_r) > 0
    runs, k, n = [], 0, act.shape[0]
    while k < n:
        if act[k]:
            e = k
            while e < n and act[e]:
                e += 1
            runs.append([k, e])
            k = e
        else:
            k += 1
    joined = []
    for s, e in (r for r in runs if r[1] - r[0] >= MINSPEECH):
        if joined and s - joined[-1][1] < JOIN:
            joined[-1][1] = e
        else:
            joined.append([s, e])
    utt = [(s, e) for s, e in joined if e - s >= MINUTT]
    if len(utt) > MAXU:
        utt = utt[:MAXU - 1] + [(utt[MAXU - 1][0], utt[-1][1])]
    return utt


def region_starts(utt: list, L: int) -> list:
    """Step 5: R_0 .. R_U (samples) of the utterances' regions."""
    if not utt:
        return [0, L]
    return [0] + [FRAME * ((utt[u - 1][1] + utt[u][0]) // 2) for u in range(1, len(utt))] + [L]


def crude_window(env_r: np.ndarray, env_d: np.ndarray, k0: int, k1: int, jlo: int, jhi: int) -> int | None:
    """Step 6: lag (frames, jlo <= j <= jhi) of the largest positive correlation over reference
    frames [k0, k1)."""
    nfr = min(env_r.shape[0], env_d.shape[0])
    best, arg = 0.0, None
    for j in range(jlo, jhi + 1):
        ks, ke = max(k0, -j), min(k1, nfr - j)
        c = float(np.dot(env_r[ks:ke], env_d[ks + j:ke + j])) if ke > ks else 0.0
        if c > best:
            best, arg = c, j
    return arg


def fine_pieces(wr: np.ndarray, wd: np.ndarray, R0: int, R1: int, d0: int) -> np.ndarray:
    """Step 7: P[i][l], lag d0 - FINE + l, over piece i = [R0 + i CHUNK, min(R0 + (i+1) CHUNK, R1))."""
    L = wr.shape[0]
    m = max(1, -(-(R1 - R0) // CHUNK))
    P = np.zeros((m, 2 * FINE + 1))
    for i in range(m):
        a, b = R0 + i * CHUNK, min(R0 + (i + 1) * CHUNK, R1)
        for li, D in enumerate(range(d0 - FINE, d0 + FINE + 1)):
            lo, hi = max(a, 1, 1 - D), min(b, L, L - D)
            if hi > lo:
                P[i, li] = float(np.dot(wr[lo:hi], wd[lo + D:hi + D]))
    return P


def _peak(c: np.ndarray):
    i = int(np.argmax(c))
    return (float(c[i]), i) if c[i] > 0 else (0.0, -1)


def pick_split(P: np.ndarray, d0: int):
    """Step 8: [(piece offset, delay)] of one region: one segment, or two after a split."""
    W = P.sum(axis=0)
    vW, iW = _peak(W)
    dW = d0 - FINE + iW if iW >= 0 else d0
    m = P.shape[0]
    best = None
    if m >= 4:
        left = np.zeros_like(W)
        for s in range(1, m - 1):
            left = left + P[s - 1]
            if s < 2:
                continue
            vL, iL = _peak(left)
            vR, iR = _peak(W - left)
            if best is None or vL + vR > best[0]:
                best = (vL + vR, s, vL, iL, vR, iR)
    if best is not None:
        tot, s, vL, iL, vR, iR = best
        if vL > 0 and vR > 0 and tot > SPLIT_GAIN * vW and abs(iL - iR) >= SPLIT_MIN:
            return [(0, d0 - FINE + iL), (s * CHUNK, d0 - FINE + iR)]
    return [(0, dW)]


def segments(ref: np.ndarray, deg: np.ndarray, max_delay: int = 16000):
    """(seg_start [n+1], seg_delay [n], row delay) of one row pair (steps 5-8)."""
    r = np.asarray(ref, dtype=np.float64)
    d = np.asarray(deg, dtype=np.float64)
    L = r.shape[0]
    env_r, env_d = envelope(r), envelope(d)
    nfr = env_r.shape[0]
    M = min(-(-max_delay // FRAME), nfr - 1) if nfr >= 2 else 0
    jrow = crude_delay(env_r, env_d, -(-max_delay // FRAME)) if nfr >= 2 else 0
    utt = utterances(env_r)
    R = region_starts(utt, L)
    wr = np.zeros(L)
    wd = np.zeros(L)
    wr[1:] = np.diff(r)
    wd[1:] = np.diff(d)
    starts, delays = [], []
    wins = utt if utt else [(0, nfr)]
    for u, (s, e) in enumerate(wins):
        j = crude_window(env_r, env_d, max(0, s - SEARCHBUF), min(nfr, e + SEARCHBUF),
                         max(-M, jrow - SEARCHBUF), min(M, jrow + SEARCHBUF))
        d0 = FRAME * (j if j is not None else jrow)
        for off, D in pick_split(fine_pieces(wr, wd, R[u], R[u + 1], d0), d0):
            if delays and delays[-1] == D:
                continue  # merged with the previous segment
            starts.append(R[u] + off)
            delays.append(D)
    starts.append(L)
    lens = np.diff(starts)
    return np.array(starts), np.array(delays), int(delays[int(np.argmax(lens))])


def shift_segments(deg: np.ndarray, starts, delays) -> np.ndarray:
    """Step 9."""
    L = deg.shape[0]
    out = np.zeros_like(deg)
    for k, D in enumerate(delays):
        a, b = int(starts[k]), int(starts[k + 1])
        lo, hi = max(a, -D), min(b, L - D)
        if hi > lo:
            out[lo:hi] = deg[lo + D:hi + D]
    return out


def align_utterances(ref: np.ndarray, deg: np.ndarray, max_delay: int = 16000, lengths=None):
    """(aligned [B, L], row delays [B], [(seg_start, seg_delay)] per row) for [B, L] rows."""
    ref = np.atleast_2d(ref)
    deg = np.atleast_2d(deg)
    B, L = ref.shape
    out = np.zeros_like(deg)
    ds = np.zeros(B, dtype=np.int64)
    segs = []
    for b in range(B):
        n = L if lengths is None else int(min(max(lengths[b], 0), L))
        st, dl, ds[b] = segments(ref[b, :n], deg[b, :n], max_delay)
        out[b, :n] = shift_segments(deg[b, :n], st, dl)
        segs.append((st, dl))
    return out, ds, segs


# ----------------------------------------------------------------------------- P.862 mode
# Steps 1-7 as the utterance mode; then, per utterance region (P.862 sections 10.5-10.6 restated
# on the fine stage's 320 ms pieces instead of P.862's 64 ms frames with 75 % overlap):
#
# 10. Piece peaks: piece i's first maximum of its first-difference correlation over the lags,
#     (v_i, l_i) when v_i > 0 (P.862 ``time_align``: each frame's cross-correlation peak).  A
#     piece votes when v_i >= REL_MIN times the utterance's largest piece peak: the regions
#     include the gaps around an utterance, whose noise-only pieces would otherwise vote with
#     weights close to the speech pieces' (the 1/8 power compresses 1e-4 to 0.32 against 1.4 for
#     a speech piece) -- P.862 takes only the utterance's frames.
# 11. Histogram delay of a range of pieces [a, b) (P.862 10.5): H[l] = sum of v_i^0.125 over the
#     range's voting pieces peaking at lag l; S = H smoothed by the triangle (T + 1 - |k|),
#     |k| <= T; the delay is the first maximum of S, its confidence S_max / ((T + 1) sum H) in
#     (0, 1]; a range without a voting piece keeps the utterance's crude delay, confidence 0.
# 12. Recursive split (P.862 10.6 ``utterance_split``, to depth MAXDEPTH): a range of >= 4 pieces
#     is tried at every piece boundary s in [a + 2, b - 2]; a candidate's two halves must each hold
#     >= 2 voting pieces, differ in delay by >= SPLIT_MIN samples and both be more confident than
#     the whole range; the candidate with the largest summed confidence (first such s) splits the
#     range and each half is tried again.  Up to 2^MAXDEPTH segments per utterance, in order; the row's segments are the
#     utterances' in order, equal neighbours merged, at most MAXSEG (later ones merge into the
#     last); the row's delay is its longest segment's (the first of equals).
HIST_T = 8        # lags: half-width of the histogram's triangular smoothing (0.5 ms)
HIST_POW = 0.125  # weight of a piece: its correlation peak to this power (P.862)
REL_MIN = 0.05    # a piece votes from this fraction of the utterance's largest piece peak
MAXDEPTH = 2


def piece_peaks(P: np.ndarray):
    """Step 10: ([m] peak values, [m] peak lag indices; -1 where the piece does not vote)."""
    v = np.zeros(P.shape[0])
    idx = np.full(P.shape[0], -1, dtype=np.int64)
    for i in range(P.shape[0]):
        j = int(np.argmax(P[i]))
        if P[i, j] > 0:
            v[i], idx[i] = P[i, j], j
    vmax = v.max() if v.size else 0.0
    idx[v < REL_MIN * vmax] = -1
    return v, idx


def hist_delay(v: np.ndarray, idx: np.ndarray, a: int, b: int, d0: int):
    """Step 11: (delay, confidence, voting pieces) of pieces [a, b)."""
    H = np.zeros(2 * FINE + 1)
    nv = 0
    for i in range(a, b):
        if idx[i] >= 0:
            H[idx[i]] += v[i] ** HIST_POW
            nv += 1
    tot = H.sum()
    if nv == 0:
        return d0, 0.0, 0
    S = np.zeros_like(H)
    for k in range(-HIST_T, HIST_T + 1):
        w = HIST_T + 1 - abs(k)
        if k >= 0:
            S[:H.shape[0] - k] += w * H[k:]
        else:
            S[-k:] += w * H[:H.shape[0] + k]
    j = int(np.argmax(S))
    return d0 - FINE + j, float(S[j] / ((HIST_T + 1) * tot)), nv


def split_p862(v, idx, a: int, b: int, d0: int, depth: int = 0) -> list:
    """Step 12: [(piece offset from a, delay)] of pieces [a, b)."""
    D, c, _ = hist_delay(v, idx, a, b, d0)
    if depth < MAXDEPTH and b - a >= 4:
        best = None
        for s in range(a + 2, b - 1):
            if b - s < 2:
                break
            dL, cL, nL = hist_delay(v, idx, a, s, d0)
            dR, cR, nR = hist_delay(v, idx, s, b, d0)
            if (nL >= 2 and nR >= 2 and abs(dL - dR) >= SPLIT_MIN and cL > c and cR > c
                    and (best is None or cL + cR > best[0])):
                best = (cL + cR, s)
        if best is not None:
            s = best[1]
            return (split_p862(v, idx, a, s, d0, depth + 1) +
                    [(s - a + o, d) for o, d in split_p862(v, idx, s, b, d0, depth + 1)])
    return [(0, D)]


def segments_p862(ref: np.ndarray, deg: np.ndarray, max_delay: int = 16000):
    """(seg_start [n+1], seg_delay [n], row delay) of one row pair (steps 5-7, 10-12)."""
    r = np.asarray(ref, dtype=np.float64)
    d = np.asarray(deg, dtype=np.float64)
    L = r.shape[0]
    env_r, env_d = envelope(r), envelope(d)
    nfr = env_r.shape[0]
    M = min(-(-max_delay // FRAME), nfr - 1) if nfr >= 2 else 0
    jrow = crude_delay(env_r, env_d, -(-max_delay // FRAME)) if nfr >= 2 else 0
    utt = utterances(env_r)
    R = region_starts(utt, L)
    wr = np.zeros(L)
    wd = np.zeros(L)
    wr[1:] = np.diff(r)
    wd[1:] = np.diff(d)
    starts, delays = [], []
    wins = utt if utt else [(0, nfr)]
    for u, (s, e) in enumerate(wins):
        j = crude_window(env_r, env_d, max(0, s - SEARCHBUF), min(nfr, e + SEARCHBUF),
                         max(-M, jrow - SEARCHBUF), min(M, jrow + SEARCHBUF))
        d0 = FRAME * (j if j is not None else jrow)
        v, idx = piece_peaks(fine_pieces(wr, wd, R[u], R[u + 1], d0))
        for off, D in split_p862(v, idx, 0, v.shape[0], d0):
            if delays and delays[-1] == D:
                continue  # merged with the previous segment
            if len(delays) == MAXSEG:
                continue  # the row's segment table is full: the last segment runs on
            starts.append(R[u] + off * CHUNK)
            delays.append(D)
    starts.append(L)
    lens = np.diff(starts)
    return np.array(starts), np.array(delays), int(delays[int(np.argmax(lens))])


def align_p862(ref: np.ndarray, deg: np.ndarray, max_delay: int = 16000, lengths=None):
    """(aligned [B, L], row delays [B], [(seg_start, seg_delay)] per row) for [B, L] rows."""
    ref = np.atleast_2d(ref)
    deg = np.atleast_2d(deg)
    B, L = ref.shape
    out = np.zeros_like(deg)
    ds = np.zeros(B, dtype=np.int64)
    segs = []
    for b in range(B):
        n = L if lengths is None else int(min(max(lengths[b], 0), L))
        st, dl, ds[b] = segments_p862(ref[b, :n], deg[b, :n], max_delay)
        out[b, :n] = shift_segments(deg[b, :n], st, dl)
        segs.append((st, dl))
    return out, ds, segs


# ----------------------------------------------------------------------------- bad intervals
# P.862 realigns "bad intervals" after its perceptual model (section 10.7, restated): with the
# segment-aligned degraded row scored,
# 13. bad frames are those whose symmetric frame disturbance exceeds BAD_THR (P.862's
#     THRESHOLD_BAD_FRAMES); runs of them closer than BAD_GAP frames join, intervals from BAD_MIN
#     frames are kept (at most MAXBAD per row, in order);
# 14. each interval's samples [256 f0, 256 f1 + 256) get the first-difference correlation's first
#     maximum within +-FINE of the delay of the segment holding sample 256 f0 (that delay if no lag
#     correlates positively), and a second degraded row takes those samples at that delay;
# 15. the second row is scored too, and an interval's frames take its symmetric and asymmetric
#     disturbances when their symmetric sum over the interval is smaller (P.862 keeps the better
#     alignment of a bad interval); the MOS pools the combined frames as PESQ.py:168-172, 240-243.
BAD_THR = 30.0
BAD_GAP = 4
BAD_MIN = 5
MAXBAD = 16
HOP = 256


def bad_intervals(sym: np.ndarray) -> list:
    """Step 13: [(f0, f1)] frames of one row's bad intervals."""
    bad = np.asarray(sym) > BAD_THR
    runs, f, n = [], 0, bad.shape[0]
    while f < n:
        if bad[f]:
            e = f
            while e < n and bad[e]:
                e += 1
            if runs and f - runs[-1][1] < BAD_GAP:
                runs[-1][1] = e
            else:
                runs.append([f, e])
            f = e
        else:
            f += 1
    return [(a, b) for a, b in runs if b - a >= BAD_MIN][:MAXBAD]


def interval_delay(ref: np.ndarray, deg: np.ndarray, a: int, b: int, d0: int) -> int:
    """Step 14: the interval's delay over samples [a, b) within +-FINE of d0."""
    r = np.asarray(ref, dtype=np.float64)
    d = np.asarray(deg, dtype=np.float64)
    L = r.shape[0]
    wr = np.zeros(L)
    wd = np.zeros(L)
    wr[1:] = np.diff(r)
    wd[1:] = np.diff(d)
    best, arg = 0.0, d0
    for D in range(d0 - FINE, d0 + FINE + 1):
        lo, hi = max(a, 1, 1 - D), min(b, L, L - D)
        if hi <= lo:
            continue
        c = float(np.dot(wr[lo:hi], wd[lo + D:hi + D]))
        if c > best:
            best, arg = c, D
    return arg


def realign_bad(ref, deg, aligned, seg_start, seg_delay, sym):
    """Step 14 for one row: ([(f0, f1, delay)], the second degraded row)."""
    L = deg.shape[0]
    out = np.array(aligned, copy=True)
    res = []
    for f0, f1 in bad_intervals(sym):
        a, b = HOP * f0, min(HOP * f1 + HOP, L)
        k = int(np.searchsorted(seg_start, a, side="right")) - 1
        D = interval_delay(ref, deg, a, b, int(seg_delay[k]))
        res.append((f0, f1, D))
        for n in range(a, b):
            out[n] = deg[n + D] if 0 <= n + D < L else 0.0
    return res, out


def pesq_p862(ref: np.ndarray, deg: np.ndarray, max_delay: int = 16000):
    """(MOS [B], [[(f0, f1, delay)] per row]) of [B, L] rows: P.862-mode alignment, then the
    bad-interval realignment (steps 13-15) on the oracle's PESQ model."""
    from oracle import pesq_oracle as po
    ref = np.atleast_2d(ref).astype(np.float32)
    deg = np.atleast_2d(deg).astype(np.float32)
    aligned, _, segs = align_p862(ref, deg, max_delay)
    i1, i2 = {}, {}
    po.disturbances(ref, aligned, i1)
    s1, a1 = i1["sym_frame"].copy(), i1["asym_frame"].copy()
    second = np.array(aligned, copy=True)
    bad = []
    for b in range(ref.shape[0]):
        res, second[b] = realign_bad(ref[b], deg[b], aligned[b], segs[b][0], segs[b][1], s1[b])
        bad.append(res)
    po.disturbances(ref, second, i2)
    s2, a2 = i2["sym_frame"], i2["asym_frame"]
    for b, res in enumerate(bad):
        for f0, f1, _ in res:
            if s2[b, f0:f1].sum() < s1[b, f0:f1].sum():
                s1[b, f0:f1] = s2[b, f0:f1]
                a1[b, f0:f1] = a2[b, f0:f1]
    return po.mos_from_distances(po.overlapping_sums(s1), po.overlapping_sums(a1)), bad
