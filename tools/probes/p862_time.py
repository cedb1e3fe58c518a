"""Time PESQ(time_align="p862") (alignment + frames + bad-interval realignment + second frames +
pooling) against plain PESQ on the gated rows of tests/align_cases.py at B x 10 s.
Usage: python tools/probes/p862_time.py [B]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from fast_speech_enhancement_metrics_amd import PESQ  # noqa: E402
from tests import align_cases as AC  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
L = 160000
base = [AC.gated_pair(900 + b, L, [(30000, 33000, 450), (90000, 93000, -100)]) for b in range(16)]
c = torch.from_numpy(np.stack([base[b % 16][0] for b in range(B)])).cuda()
d = torch.from_numpy(np.stack([base[b % 16][1] for b in range(B)])).cuda()
out = {"batch": B, "length": L}
for name, m in (("pesq", PESQ(16000, use_gpu=True)), ("p862", PESQ(16000, use_gpu=True, time_align="p862")),
                ("utterance", PESQ(16000, use_gpu=True, time_align="utterance"))):
    m.scores(c, d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        r = m.scores(c, d)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 3 * 1e3
    out[name] = {"ms": round(ms, 2), "utt_per_s": round(B / ms * 1e3, 1), "mean_mos": float(r.float().mean())}
m = PESQ(16000, use_gpu=True, time_align="p862")
_, _, nb, _ = m.p862_scores(c, d)
out["rows_with_intervals"] = int((nb > 0).sum())
print(json.dumps(out))
