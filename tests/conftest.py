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
    # the test run opts in to rebuilding a stale engine (the package itself refuses one unless
    # FSEM_AUTOBUILD=1, _native._check_build_id); a no-op when libfsem.so matches the tree
    from fast_speech_enhancement_metrics_amd import _build
    if _build._stale():
        try:
            _build.build()
        except RuntimeError:  # no hipcc: the tests that load the engine fail with its message
            pass


def load_golden(name: str):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    out = {k: d[k] for k in d.files}
    if "clean_f32" in out:  # float32 rows stored as such (inputs off the int16 grid)
        out["clean_f"], out["noisy_f"] = out["clean_f32"], out["noisy_f32"]
        return out
    out["clean_f"] = out["clean"].astype(np.float32) / 32768.0
    out["noisy_f"] = out["noisy"].astype(np.float32) / 32768.0
    return out


def edge_inputs(g, name: str):
    """(clean, noisy) float32 tensors of edge case `name` of the edges_16k golden, rebuilt exactly as
    tests/golden/make_golden.py fed them to the reference: codes / 32768 * scale + offset."""
    import torch
    k = list(g["names"]).index(name)
    sc, oc, on = (float(v) for v in g["params"][k])
    c = torch.from_numpy(g["clean"]).to(torch.float32) / 32768.0
    n = torch.from_numpy(g["noisy"]).to(torch.float32) / 32768.0
    scale = torch.tensor(sc, dtype=torch.float32)
    return c * scale + torch.tensor(oc, dtype=torch.float32), n * scale + torch.tensor(on, dtype=torch.float32)


PESQ_CASES = ["pesq_3s", "pesq_ragged", "pesq_10s", "pesq_hi_snr", "pesq_lo_snr", "pesq_wide"]
STOI_CASES = ["stoi_10k", "stoi_16k", "stoi_16k_10s", "stoi_wide"]


@pytest.fixture(params=PESQ_CASES)
def pesq_golden(request):
    return load_golden(request.param)


@pytest.fixture(params=STOI_CASES)
def stoi_golden(request):
    return load_golden(request.param)
