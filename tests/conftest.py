import os
import sys

import numpy as np
import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name: str):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    out = {k: d[k] for k in d.files}
    out["clean_f"] = out["clean"].astype(np.float32) / 32768.0
    out["noisy_f"] = out["noisy"].astype(np.float32) / 32768.0
    return out


PESQ_CASES = ["pesq_3s", "pesq_ragged", "pesq_10s", "pesq_hi_snr", "pesq_lo_snr", "pesq_wide"]
STOI_CASES = ["stoi_10k", "stoi_16k", "stoi_16k_10s", "stoi_wide"]


@pytest.fixture(params=PESQ_CASES)
def pesq_golden(request):
    return load_golden(request.param)


@pytest.fixture(params=STOI_CASES)
def stoi_golden(request):
    return load_golden(request.param)
