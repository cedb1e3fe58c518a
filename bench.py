#!/usr/bin/env python3
"""Benchmark: utterances/sec of PESQ-wb + STOI/ESTOI on 10 s @ 16 kHz pairs (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--length L]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = the drop-in call ``PESQ_STOI(16000, use_gpu=True)(clean, noisy)`` on this rank's batch
(4096 pairs per GPU by default: BASELINE.json configs[1], 10 s @ 16 kHz fp32) -> the list of
{"PESQ", "STOI", "ESTOI"} dicts, timed as the reference times its metrics
(benchmark_metrics.py:72-75: wall clock around ``metric(clean, noisy)``, list building included).
The call runs the fused joint entry fsem_pesq_stoi_f32 (one read of the inputs; scores bitwise
equal to the two separate API calls; ``--separate`` runs ``PESQ(...)`` + ``STOI(...)`` instead).
With N > 1 ranks every rank also all-gathers the job's [B, 3] scores over RCCL (xGMI).
``scores_path`` reports the engine API alone (``PESQ_STOI.scores`` + one device->host copy).
Weak scaling: every rank owns its own shard of utterances, generated in HBM before timing.

``--gpus N`` without a torch.distributed launcher starts the N ranks itself (a child
``torch.distributed.run`` process, before this process touches the GPU); N above the visible
device count is an error.  This one-process-per-GPU form is what the driver's scaling runs time.
``--gpus N --single-process`` times the other multi-device form instead: one process driving N
devices through ``PESQ_STOI(..., devices=N)`` (multidevice.py) on a batch held by device 0, the
shards' peer copies included.

Rank 0 prints ONE JSON line with the metric, the roofline of the dominant kernel
(pesq_front<joint>: algorithmic bytes / its HIP-event-timed duration vs 8 TB/s), the CPU
baseline (the package's use_gpu=False path on the host's cores at batch 4 and 64, as
SURVEY.md 8(d) / BASELINE.md ask) and the oracle CPU restatement beside it (``cpu_oracle``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "utterances/sec PESQ-wb+STOI, 10s@16kHz, batch 4096, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK = 157.3e12  # MI355X_MICROARCH.md: FP32 vector (= f32 MFMA) peak, FLOP/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps: the engine's step time settles over ~5 steps after the first "
                         "(workspace allocation, clocks)")
    ap.add_argument("--batch", type=int, default=4096, help="utterance pairs per GPU")
    ap.add_argument("--length", type=int, default=160000, help="samples per utterance (16 kHz)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="oracle CPU leg time budget")
    ap.add_argument("--cpu-calls", type=int, default=7, help="CPU-baseline calls per batch size")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=5)
    ap.add_argument("--separate", action="store_true", help="two API calls (PESQ, STOI) instead of the joint entry")
    ap.add_argument("--device-list", default=None,
                    help="with --single-process: explicit device indices, e.g. 0,0 (repeats allowed: "
                         "several streams on one device -- the 1-GPU rehearsal of the fan-out path)")
    ap.add_argument("--single-process", action="store_true",
                    help="with --gpus N: ONE process drives the N devices (devices=N on the metric, "
                         "multidevice.py) on a batch of N x --batch rows held by device 0 -- the timed "
                         "call includes the peer copies of the other devices' shards over xGMI")
    ap.add_argument("--workload", default="c2",
                    choices=["c2", "pesq", "pesq_aligned", "pesq_aligned_utt", "pesq_aligned_p862", "c3", "c5"],
                    help="c2: BASELINE metric (default, PESQ-wb + STOI/ESTOI); pesq: configs[1] as stated, "
                         "PESQ-wb only; c3: STOI+ESTOI only, 8192 x 5 s @ 16 kHz per GPU; "
                         "c5: config 5, mixed 8/16 kHz ragged 2-30 s batch")
    return ap.parse_args()


def cpu_oracle(clean, noisy, budget_s):
    """Oracle CPU restatement (oracle/), one core, on a bounded sample of the same workload."""
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    from oracle import pesq_oracle, stoi_oracle

    ctx = threadpool_limits(limits=1) if threadpool_limits else None
    torch_threads = torch.get_num_threads()
    torch.set_num_threads(1)
    n = 0
    t0 = time.perf_counter()
    try:
        if ctx:
            ctx.__enter__()
        while True:
            c = clean[n:n + 1].cpu().numpy()
            d = noisy[n:n + 1].cpu().numpy()
            pesq_oracle.pesq(c, d)
            stoi_oracle.stoi(c, d, 16000)
            n += 1
            if time.perf_counter() - t0 >= budget_s or n >= clean.shape[0]:
                break
    finally:
        if ctx:
            ctx.__exit__(None, None, None)
        torch.set_num_threads(torch_threads)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "utterances/s", "cores": 1, "kind": "port",
            "sample": f"{n} pairs x {clean.shape[1]} samples @16kHz, PESQ-wb + STOI/ESTOI, "
                      f"oracle numpy/C restatement, {dt:.1f} s"}


def host_cores():
    """Threads of the host's share: OMP_NUM_THREADS where the launcher sets it (16 per GPU on the
    MI355X boxes, whose os.cpu_count() is the whole machine), else every core."""
    return max(1, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(clean, noisy, batches=(4, 64), calls=7):
    """The contract's CPU baseline: the package's use_gpu=False path -- the reference's CPU mode
    restated in torch/scipy (_cpu.py) -- called as the drop-in ``PESQ_STOI(16000, use_gpu=False)
    (clean, noisy)`` on `batches` pairs of the workload, on the host's cores
    (``torch.set_num_threads``); per batch size the median of the calls left after dropping the
    first int(0.15 n) + 1 (benchmark_metrics.py:82).  value = the largest batch's rate."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    m = PESQ_STOI(16000, use_gpu=False)
    prev = torch.get_num_threads()
    threads = host_cores()
    torch.set_num_threads(threads)
    out = {}
    try:
        for b in batches:
            c, d = clean[:b].cpu(), noisy[:b].cpu()
            ts = []
            for _ in range(calls):
                t0 = time.perf_counter()
                m(c, d)
                ts.append(time.perf_counter() - t0)
            kept = sorted(ts[int(calls * 0.15) + 1:])
            med = kept[len(kept) // 2]
            out[b] = {"value": b / med, "ms_per_call": round(med * 1e3, 1), "calls": len(kept)}
    finally:
        torch.set_num_threads(prev)
    big = max(batches)
    return {"value": out[big]["value"], "unit": "utterances/s", "cores": threads, "kind": "port",
            "sample": (f"use_gpu=False drop-in call PESQ_STOI(16000)(clean, noisy) -> list of dicts, "
                       f"{clean.shape[1]} samples @16kHz, batch {big} (batch {min(batches)}: "
                       f"{out[min(batches)]['value']:.1f} utt/s), median of {out[big]['calls']} calls after "
                       f"dropping the first {calls - out[big]['calls']}; {threads} threads of {os.cpu_count()} "
                       f"logical CPUs ({cpu_model()})"),
            "batches": {str(b): v for b, v in out.items()}}


def kernel_roofline(clean, noisy, reps, joint, config_batch=None):
    """HIP-event timing of the dominant kernel -- pesq_front, launched alone through its stage
    entry (fsem_pesq_front_y10_f32 for the joint path, fsem_pesq_front_f32 otherwise) -- on the
    stream it is launched on, over the rows one engine call of the step processes (the drop-in
    call's rows per engine call, joint.chunk_bounds: all 4096); achieved = algorithmic bytes per launch / avg duration.
    `config_batch`: the bench configuration's batch (the PMC summaries are recorded at it)."""
    from fast_speech_enhancement_metrics_amd import _native
    lib = _native.load()
    B, L = clean.shape
    F = lib.fsem_pesq_frames(L)
    dev = clean.device
    bark = torch.empty(2 * B, 49, (F + 31) // 32 * 32, device=dev)  # band-major rows (include/fsem.h)
    power = torch.empty(2 * B, device=dev)
    ws = _native.workspace(lib.fsem_pesq_front_workspace_bytes(B, L), dev)
    stream = torch.cuda.current_stream(dev)
    h = stream.cuda_stream
    y_ld = ((5 * L + 7) // 8 + 63) // 64 * 64
    y10 = torch.empty(2 * B, y_ld, device=dev) if joint else None
    v_ld = (((5 * L + 7) // 8) // 64 + 1 + 63) // 64 * 64
    vad = torch.empty(B, v_ld, 2, device=dev) if joint else None  # STOI VAD quarter sums, as in the joint path

    def launch():
        if joint:
            rc = lib.fsem_pesq_front_y10_f32(clean.data_ptr(), noisy.data_ptr(), B, L, L, None, bark.data_ptr(),
                                             power.data_ptr(), y10.data_ptr(), y_ld, vad.data_ptr(), v_ld,
                                             ws.data_ptr(), ws.numel(), h)
        else:
            rc = lib.fsem_pesq_front_f32(clean.data_ptr(), noisy.data_ptr(), B, L, L, None, bark.data_ptr(),
                                         power.data_ptr(), ws.data_ptr(), ws.numel(), h)
        _native.check(rc, "front")

    for _ in range(3):  # steady state (clocks, TLB) as inside the timed steps
        launch()
    torch.cuda.synchronize(dev)
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record(stream)
    for _ in range(reps):
        launch()
    end.record(stream)
    end.synchronize()
    ms = start.elapsed_time(end) / reps
    algo_bytes = 2 * B * L * 4  # both signals read once (2*L*4 B per pair)
    achieved = algo_bytes / (ms * 1e-3) / 1e9
    name = FRONT_KERNELS[joint]
    summary, source = pmc_summary_for(_native.build_id(), B, L)
    d = pmc_kernel(summary, name)
    traffic = int(d["hbm_bytes"]) if "hbm_bytes" in d else None
    out = {"kernel": "pesq_front<joint>" if joint else "pesq_front", "bound": None, "achieved": round(achieved, 1),
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
           "traffic_source": source, "library_build_id": _native.build_id(), "ms_per_launch": round(ms, 4),
           "algorithmic_bytes_per_launch": algo_bytes}
    sims = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
    cus = sims // 4
    # what limits the kernel, from its counters (the PMC summary of THIS library build) at the
    # measured launch time: the HBM share of its counted traffic, the vector-ALU issue share
    # (SQ_INSTS_VALU x 2 cycles per wave64 instruction on a SIMD-32, MI355X_MICROARCH.md, over
    # the SIMDs x the launch time at the 2.4 GHz peak clock), the LDS-array share
    # (SQ_LDS_IDX_ACTIVE over the CUs x the launch's cycles) and the matrix pipe's
    # (SQ_INSTS_MFMA... not collected: MFMA time is < the VALU's here)
    limits = {}
    if traffic:
        limits["hbm"] = round(traffic / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 4)
    if "SQ_INSTS_VALU" in d:
        limits["valu"] = round(d["SQ_INSTS_VALU"] * 2 / (sims * 2.4e9 * ms * 1e-3), 4)
        out["valu_issue"] = {"instructions_per_launch": int(d["SQ_INSTS_VALU"]), "frac": limits["valu"],
                             "source": source}
    if "SQ_LDS_IDX_ACTIVE" in d:
        limits["lds"] = round(d["SQ_LDS_IDX_ACTIVE"] / (cus * 2.4e9 * ms * 1e-3), 4)
    if "SQ_WAIT_INST_ANY" in d and d.get("SQ_WAVE_CYCLES"):
        # issue stalls on dependencies (mfma RAW, pipe) over the waves' lifetime (MI355X_MICROARCH.md
        # 'rocprofv3 PMC slots'; SQ_WAIT_ANY = parked at s_waitcnt / barriers, the rest issuing)
        limits["wait_inst_share"] = round(d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"], 4)
        if "SQ_WAIT_ANY" in d:
            limits["wait_any_share"] = round(d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"], 4)
    if "waves_per_simd" in d:
        # achieved occupancy: mean resident waves per SIMD over the launch (tools/pmc_summary.py:
        # 4 x SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)); 2 is this kernel's limit
        out["occupancy"] = {"waves_per_simd": round(d["waves_per_simd"], 3), "limit": 2, "source": source}
    out["limits"] = limits
    out["bound"] = derive_bound(limits)
    return out


def derive_bound(limits: dict) -> str:
    """The roofline's `bound` from the counters: the resource whose share of the launch time is
    largest among HBM traffic, VALU issue and the LDS array, if that share reaches 0.6 (a pipe
    that busy is the limit); otherwise "latency" -- no pipe is near its peak and the kernel's
    time goes to dependency chains, memory round trips and barriers.  "unmeasured" without a PMC
    summary of this library build."""
    shares = {k: limits[k] for k in ("hbm", "valu", "lds") if k in limits}
    if not shares:
        return "unmeasured"
    k = max(shares, key=shares.get)
    return k if shares[k] >= 0.6 else "latency"


def step_roofline(B: int, L: int, ms_per_step: float) -> dict:
    """Step-level roofline of the timed drop-in call: SURVEY 8(d)'s algorithmic bytes per step
    (both inputs read once + 12 B of scores per pair) against HBM peak, and its informational
    FLOPs (~23 MFLOP PESQ + ~30 MFLOP STOI per 10 s pair, scaled by length) against the FP32
    vector peak (157.3 TFLOP/s, MI355X_MICROARCH.md)."""
    byts = B * (2 * L * 4 + 12)
    flops = B * 53e6 * (L / 160000)
    s = ms_per_step * 1e-3
    return {"algorithmic_bytes": byts, "hbm_achieved_gbs": round(byts / s / 1e9, 1),
            "hbm_frac": round(byts / s / (HBM_PEAK_GBS * 1e9), 4), "flops": int(flops),
            "fp32_achieved_tflops": round(flops / s / 1e12, 2), "fp32_frac": round(flops / s / FP32_PEAK, 4),
            "ms_per_step": round(ms_per_step, 3)}


# the uniform-length front-end instance in the PMC summaries' kernel names (joint / PESQ alone):
# <JOINT, VARLEN, SAFE> from round 3 on, <JOINT, VARLEN> before
FRONT_KERNELS = {True: ("pesq_front<true, false, false>", "pesq_front<true, false>"),
                 False: ("pesq_front<false, false, false>", "pesq_front<false, false>")}


def pmc_summary_for(build_id: str, rows: int, L: int):
    """(summary, source) of the committed PMC summary (profiles/*/pmc_summary.json,
    tools/pmc_summary.py) recorded on the library build `build_id` at `rows` x `L` per engine
    call (its "_meta"), or ({}, reason).  Chosen by what was measured -- the build id of the
    profiled library and the launch size -- never by directory names.  FETCH_SIZE x2 (gfx950
    correction) + WRITE_SIZE per MI355X_MICROARCH.md 'HBM'; the counters need their own rocprofv3
    passes, so they cannot be read inside the timed run."""
    import glob
    found = []
    for f in glob.glob(os.path.join(HERE, "profiles", "*", "pmc_summary*.json")):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        m = d.get("_meta", {})
        if (m.get("build_id"), m.get("rows_per_launch"), m.get("length")) == (build_id, rows, L):
            found.append((os.path.relpath(f, HERE), d))
    if not found:
        return {}, f"none: no committed PMC summary of library build {build_id} at {rows} x {L}"
    found.sort(key=lambda x: x[0])
    src, d = found[0]
    return d, src + (f" (+{len(found) - 1} more of this build)" if len(found) > 1 else "")


def pmc_kernel(summary: dict, kernel) -> dict:
    """The counters of `kernel` (a name suffix, or a tuple of them) in a PMC summary, or {}."""
    names = kernel if isinstance(kernel, tuple) else (kernel,)
    for k, v in summary.items():
        if isinstance(v, dict) and any(k.endswith(n) for n in names):
            return v
    return {}


def _timed(step, args, dev, distributed):
    for _ in range(args.warmup):
        step()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def run_c3(args, world, rank, dev, distributed):
    """BASELINE.json configs[2]: STOI+ESTOI of 8192 x 5 s @ 16 kHz pairs per GPU (fused 16->10 kHz)."""
    from fast_speech_enhancement_metrics_amd import STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    B, L = 8192, 80000
    cs, ns = [], []
    for lo in range(0, B, 2048):
        c, n, _ = speech_like_pairs(2048, L, 16000, seed=77 + 13 * rank + lo, device=dev)
        cs.append(c)
        ns.append(n)
    clean, noisy = torch.cat(cs), torch.cat(ns)
    del cs, ns
    stoi = STOI(16000, use_gpu=True)

    def step():
        s, e = stoi.scores(clean, noisy, 16000)
        local = torch.stack([s, e], 1)
        return local.cpu() if rank == 0 else None

    dt = _timed(step, args, dev, distributed)
    if rank == 0:
        print(json.dumps({
            "metric": "utterances/sec STOI+ESTOI, 5s@16kHz, batch 8192 (config 3)",
            "value": round(world * B * args.steps / dt, 2), "unit": "utterances/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic speech-like pairs",
            "config": {"workload": "config 3: STOI/ESTOI scores, fused 16->10 kHz resampling",
                       "batch_per_gpu": B, "length": L, "sample_rate": 16000,
                       "parallelism": f"dp{world}"}}), flush=True)


def run_pesq(args, world, rank, dev, distributed):
    """BASELINE.json configs[1] as stated there: PESQ-wb alone, 4096 x 10 s @ 16 kHz pairs per GPU
    (PESQ.scores: front end, signal powers folded into the back end, back end).  The headline
    metric (default workload) adds STOI/ESTOI through the joint entry."""
    from fast_speech_enhancement_metrics_amd import PESQ
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    B, L = 4096, 160000
    clean, noisy, _ = speech_like_pairs(B, L, 16000, seed=42 + rank, device=dev)
    aligned = args.workload in ("pesq_aligned", "pesq_aligned_utt", "pesq_aligned_p862")
    mode = {"pesq_aligned_utt": "utterance", "pesq_aligned_p862": "p862"}.get(args.workload, "row")
    if aligned:
        # extension (not in the reference): degraded rows delayed by U[-2000, 2000] samples,
        # PESQ(time_align=True) estimates and undoes the delay before scoring (alignment.py)
        g = torch.Generator(device=dev)
        g.manual_seed(7 + rank)
        delay = torch.randint(-2000, 2001, (B,), generator=g, device=dev)
        src = torch.arange(L, device=dev)[None, :] - delay[:, None]
        noisy = torch.where((src >= 0) & (src < L), noisy.gather(1, src.clamp(0, L - 1)), torch.zeros_like(noisy))
        del src
    pesq = PESQ(16000, use_gpu=True, time_align=mode if aligned else False)

    def step():
        p = pesq.scores(clean, noisy)
        return p.cpu() if rank == 0 else None

    dt = _timed(step, args, dev, distributed)
    if aligned:
        found = int((pesq.last_delays.long() == delay).sum())
    if rank == 0:
        line = {
            "metric": (f"utterances/sec PESQ-wb with time alignment ({mode} mode, extension), 10s@16kHz, batch 4096"
                       if aligned
                       else "utterances/sec PESQ-wb, 10s@16kHz, batch 4096 (config 2)"),
            "value": round(world * B * args.steps / dt, 2), "unit": "utterances/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic speech-like pairs" + (", degraded rows delayed by U[-2000, 2000] samples" if aligned
                                                     else ""),
            "config": {"workload": (f"PESQ(16000, use_gpu=True, time_align={mode!r}).scores" if aligned
                                    else "config 2: PESQ-wb scores (PESQ.scores)"), "batch_per_gpu": B,
                       "length": L, "sample_rate": 16000, "parallelism": f"dp{world}"}}
        if aligned:
            line["delays_recovered"] = f"{found}/{B}"
        print(json.dumps(line), flush=True)


def run_c5(args, world, rank, dev, distributed):
    """BASELINE.json configs[4] / SURVEY 8(d) C5: 2048 utterances per GPU (16384 on 8), lengths
    uniform in 2-30 s, half at 8 kHz (PESQ via 8->16 kHz, STOI via 8->10 kHz, as the reference's
    PESQ(8000) / STOI(8000)) and half at 16 kHz (joint entry); ragged rows with per-row lengths.
    The global plan (lengths, rates) is seeded and identical on every rank; utterances go to
    ranks by LPT over their 16 kHz-equivalent length (distributed.lpt_shards)."""
    import numpy as np
    from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
    from fast_speech_enhancement_metrics_amd.distributed import lpt_shards
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs

    n_total = 2048 * world
    rng = np.random.default_rng(5)
    secs = rng.uniform(2.0, 30.0, size=n_total)
    rate = np.where(np.arange(n_total) % 2 == 0, 8000, 16000)
    lens = np.round(secs * rate).astype(np.int64)
    cost = np.where(rate == 8000, 2 * lens, lens)  # 16 kHz-equivalent samples
    mine = np.array(lpt_shards(cost, world)[rank], dtype=np.int64)
    groups = {}
    for sr in (8000, 16000):
        idx = mine[rate[mine] == sr]
        ln = lens[idx]
        cap = int(-(-int(ln.max()) // 4) * 4)
        cs, ns = [], []
        for lo in range(0, len(idx), 256):  # generate in slices (bounded temporaries)
            c, n, _ = speech_like_pairs(min(256, len(idx) - lo), cap, sr, seed=1000 + 7 * rank + lo + sr, device=dev)
            cs.append(c)
            ns.append(n)
        groups[sr] = (torch.cat(cs), torch.cat(ns), torch.from_numpy(ln.astype(np.int32)).to(dev))
    joint = PESQ_STOI(16000, use_gpu=True)
    p8, s8 = PESQ(8000, use_gpu=True), STOI(8000, use_gpu=True)

    def step():
        c, n, l16 = groups[16000]
        out16 = torch.stack(joint.scores(c, n, lengths=l16), 1)
        c8, n8, l8 = groups[8000]
        mos8 = p8.scores(c8, n8, lengths=l8, sample_rate=8000)  # 8 -> 16 kHz, each row as the row alone
        st8, es8 = s8.scores(c8, n8, 8000, lengths=l8)
        out8 = torch.stack([mos8, st8, es8], 1)
        res = torch.cat([out8, out16])
        return res.cpu() if rank == 0 else None

    dt = _timed(step, args, dev, distributed)
    if rank == 0:
        audio_s = float(secs.sum())
        print(json.dumps({
            "metric": "utterances/sec PESQ+STOI, mixed 8/16 kHz, variable 2-30 s (config 5)",
            "value": round(n_total * args.steps / dt, 2), "unit": "utterances/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic speech-like pairs, lengths U[2,30] s, half 8 kHz / half 16 kHz",
            "config": {"workload": "config 5: ragged PESQ-wb (8 kHz via 8->16 kHz) + STOI/ESTOI, per-row lengths",
                       "global_batch": n_total, "audio_seconds_per_step": round(audio_s, 1),
                       "audio_seconds_per_sec": round(audio_s * args.steps / dt, 1),
                       "parallelism": f"dp{world} (LPT shards by 16 kHz-equivalent length)"}}), flush=True)


def spawn_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N ranks as a child torch.distributed.run process (this
    process has not touched the GPU: device_count() does not initialise HIP on this image) and
    return its exit code.  N above the visible devices is an error."""
    import socket
    import subprocess
    visible = torch.cuda.device_count()
    if n > visible:
        print(f"bench.py: --gpus {n} but only {visible} HIP device(s) are visible", file=sys.stderr)
        return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def run_single_process(args):
    """--single-process: the drop-in call PESQ_STOI(16000, use_gpu=True, devices=N)(clean, noisy)
    from one process on N x --batch rows resident on device 0 (the reference user's batch on
    "cuda"): each shard is copied to its device over xGMI inside the timed call, scored there on
    its own stream, and the scores come back to device 0 (multidevice.py)."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    devices = [int(x) for x in args.device_list.split(",")] if args.device_list else list(range(args.gpus))
    n = len(devices)
    visible = torch.cuda.device_count()
    if max(devices) >= visible:
        print(f"bench.py: devices {devices} but only {visible} HIP device(s) are visible", file=sys.stderr)
        sys.exit(2)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, L = n * args.batch, args.length
    cs, ns = [], []
    for lo in range(0, B, 2048):
        c, x, _ = speech_like_pairs(min(2048, B - lo), L, 16000, seed=42 + lo, device=dev)
        cs.append(c)
        ns.append(x)
    clean, noisy = torch.cat(cs), torch.cat(ns)
    del cs, ns
    metric = PESQ_STOI(16000, use_gpu=True, devices=[f"cuda:{d}" for d in devices])

    def step():
        return metric(clean, noisy)

    dt = _timed(step, args, dev, False)
    print(json.dumps({
        "metric": METRIC + " (one process, devices=N)", "value": round(B * args.steps / dt, 2),
        "unit": "utterances/s", "n_gpus": len(set(devices)), "devices": devices, "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic speech-like pairs, the whole batch on device 0",
        "config": {"workload": "PESQ_STOI(16000, use_gpu=True, devices=N)(c, n) -> list of dicts, including the "
                               "peer copies of N-1 shards from device 0", "batch_per_gpu": args.batch,
                   "global_batch": B, "length": L, "sample_rate": 16000,
                   "parallelism": f"{n} shards on devices {devices} from one process (multidevice.py)"}}),
          flush=True)


def main():
    args = parse()
    if args.single_process:
        if args.workload != "c2":
            print(f"bench.py: --single-process times the c2 joint drop-in call only (got --workload {args.workload})",
                  file=sys.stderr)
            sys.exit(2)
        run_single_process(args)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = "WORLD_SIZE" in os.environ  # launched by torch.distributed.run (any N)
    if distributed and world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks", file=sys.stderr)
    if distributed:
        # RCCL prints a version banner on the process's stdout at init: route native stdout to
        # stderr so the result line stays the only line on stdout
        out_fd = os.dup(1)
        os.dup2(2, 1)
        sys.stdout = os.fdopen(out_fd, "w", buffering=1)
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.workload in ("pesq", "pesq_aligned", "pesq_aligned_utt", "pesq_aligned_p862", "c3", "c5"):
        {"pesq": run_pesq, "pesq_aligned": run_pesq, "pesq_aligned_utt": run_pesq, "pesq_aligned_p862": run_pesq,
         "c3": run_c3,
         "c5": run_c5}[args.workload](
            args, world, rank, dev, distributed)
        if distributed:
            dist.barrier()
            dist.destroy_process_group()
        return

    from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
    from fast_speech_enhancement_metrics_amd.distributed import gather_scores
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs

    B, L = args.batch, args.length
    clean, noisy, _ = speech_like_pairs(B, L, 16000, seed=42 + rank, device=dev)
    torch.cuda.synchronize(dev)
    pesq = PESQ(16000, use_gpu=True)
    stoi = STOI(16000, use_gpu=True)
    joint = PESQ_STOI(16000, use_gpu=True)

    def step():
        # the drop-in call on this rank's pairs -> list of dicts (the reference's measured unit)
        if args.separate:
            res = [{**a, **b} for a, b in zip(pesq(clean, noisy), stoi(clean, noisy))]
        elif distributed:
            res, local_scores = joint.call_with_scores(clean, noisy)
        else:
            res = joint(clean, noisy)
        if distributed:  # the job's scores on every rank: RCCL all-gather over xGMI
            if args.separate:
                local_scores = torch.tensor([[d["PESQ"], d["STOI"], d["ESTOI"]] for d in res], device=dev)
            gather_scores(local_scores, world * B)
        return res

    # the drop-in call's engine calls (row chunks; joint.chunk_bounds): the scores path and the
    # roofline launch the kernels at the same per-call size, so every pesq_front launch of this
    # command has one size and rocprofv3's average is the roofline's launch
    bounds = joint.chunk_bounds(B, True) if not args.separate else [(0, B)]
    launch_rows = max(hi - lo for lo, hi in bounds)

    def scores_step():
        # engine API alone: scores on the device (the same row chunks), one device->host copy
        parts = [torch.stack(joint.scores(clean[lo:hi], noisy[lo:hi]), dim=1) for lo, hi in bounds]
        local = parts[0] if len(parts) == 1 else torch.cat(parts)
        full = gather_scores(local, world * B) if distributed else local
        return full.cpu() if rank == 0 else None

    # the dominant kernel's roofline (HIP-event timed launches of its stage entry) first: the
    # GPU's clocks are still ramping during the first steps after the input generation
    roof = kernel_roofline(clean[:launch_rows], noisy[:launch_rows], args.kernel_reps, joint=not args.separate,
                           config_batch=B)
    dt = _timed(step, args, dev, distributed)
    ms_per_step = dt / args.steps * 1e3
    value = world * B * args.steps / dt
    dt_s = _timed(scores_step, args, dev, distributed)

    if rank == 0:
        cpu = oracle = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(clean, noisy, batches=tuple(sorted({min(4, B), min(64, B)})), calls=args.cpu_calls)
            oracle = cpu_oracle(clean, noisy, args.cpu_seconds)
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "utterances/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (speech-like harmonic source + AM noise, SNR U[-5,25] dB, int16 grid)",
            "config": {"workload": ("PESQ-wb + STOI/ESTOI of 10 s @ 16 kHz fp32 pairs through the drop-in call "
                                    + ("PESQ(16000)(c, n) + STOI(16000)(c, n)" if args.separate else
                                       "PESQ_STOI(16000, use_gpu=True)(c, n) (fused joint entry, one read of "
                                       "the inputs)") + " -> list of dicts"),
                       "batch_per_gpu": B, "global_batch": world * B, "length": L, "sample_rate": 16000,
                       "parallelism": f"dp{world} (utterance shards, RCCL all-gather of scores)"},
            "roofline": {**roof, "step": step_roofline(B, L, ms_per_step)}, "cpu_baseline": cpu, "cpu_oracle": oracle,
            "scores_path": {"value": round(world * B * args.steps / dt_s, 2), "unit": "utterances/s",
                            "ms_per_step": round(dt_s / args.steps * 1e3, 3),
                            "what": "PESQ_STOI.scores + one device->host copy (no list of dicts)"},
        }
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
