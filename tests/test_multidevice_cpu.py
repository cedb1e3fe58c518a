"""Host logic of the single-process multi-device path (multidevice.py): the row split
and the devices= argument's validation.  The fan-out itself runs in tests/test_multidevice_gpu.py."""
import pytest
import torch

from fast_speech_enhancement_metrics_amd.multidevice import resolve_devices, row_shards


def test_row_shards_by_count_cover_rows_in_order():
    for B in (0, 1, 5, 7, 4096):
        for n in (1, 2, 3, 8):
            b = row_shards(B, n)
            assert len(b) == n and b[0][0] == 0 and b[-1][1] == B
            assert all(b[k][1] == b[k + 1][0] for k in range(n - 1))
            sizes = [hi - lo for lo, hi in b]
            assert max(sizes) - min(sizes) <= 1


def test_row_shards_by_length_balance_contiguously():
    lengths = torch.tensor([32000, 480000, 16000, 16000, 480000, 64000, 8000, 240000], dtype=torch.int32)
    b = row_shards(8, 2, lengths)
    assert b[0][0] == 0 and b[-1][1] == 8 and b[0][1] == b[1][0]
    total = int(lengths.sum())
    prefix = [int(lengths[:j].sum()) for j in range(9)]
    # the contiguous cut is the row boundary closest to half the total
    best = min(range(9), key=lambda j: abs(prefix[j] - total / 2))
    assert b[0][1] == best
    # more shards than rows: empty shards, every row exactly once
    b = row_shards(3, 5, torch.tensor([10, 10, 10]))
    assert sum(hi - lo for lo, hi in b) == 3 and b[-1][1] == 3


def test_resolve_devices_validation():
    assert resolve_devices(None) is None
    with pytest.raises(TypeError):
        resolve_devices(1.5)
    with pytest.raises(ValueError):
        resolve_devices(0)
    with pytest.raises(ValueError):
        resolve_devices([])
    with pytest.raises(ValueError):
        resolve_devices(["cpu"])
    n = torch.cuda.device_count()
    with pytest.raises(ValueError):  # past the visible devices
        resolve_devices([f"cuda:{n}"])
    if n == 0:  # no visible device (the CPU container): "all" is an empty list
        with pytest.raises(ValueError):
            resolve_devices("all")
    else:
        assert resolve_devices("all") == [torch.device("cuda", i) for i in range(n)]


def test_cpu_metrics_ignore_devices():
    """devices= is a GPU option: a CPU-mode metric keeps the reference's CPU behaviour."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    m = PESQ_STOI(16000, use_gpu=False, devices=None)
    assert m.devices is None and not m.fans_out()
