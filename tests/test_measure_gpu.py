"""The measurement entry points bench.py builds its kernel table from (no reference counterpart):
kair_ktime_* (dispatch-packet timestamps of every libkair launch) and kair_gate_* (an eager pass queued behind a
held wave)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _axpy_burst(H, n=4):
    y = torch.zeros(1 << 22, device="cuda")
    x = torch.ones_like(y)
    for _ in range(n):
        H.axpy(y, x, 1.0)
    return y


def test_ktime_times_every_launch():
    from kair_amd import _hip as H
    torch.cuda.synchronize()
    H.ktime_begin(64)
    try:
        y = _axpy_burst(H)
    finally:
        n = H.ktime_end()
    torch.cuda.synchronize()
    assert n == 4 and H.ktime_count() == 4
    for i in range(n):
        ms, name = H.ktime_read(i)
        assert 0.0 < ms < 50.0, ms
        assert "axpy_kernel" in name, name
    assert float(y[0]) == 4.0
    # closed window: launches are not taken
    _axpy_burst(H, 1)
    assert H.ktime_count() == 4


def test_ktime_skips_capturing_streams():
    from kair_amd import _hip as H
    y = torch.zeros(1 << 16, device="cuda")
    x = torch.ones_like(y)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    H.ktime_begin(16)
    try:
        with torch.cuda.stream(s):
            g.capture_begin()
            try:
                H.axpy(y, x, 1.0)
            finally:
                g.capture_end()
    finally:
        n = H.ktime_end()
    torch.cuda.current_stream().wait_stream(s)
    assert n == 0
    g.replay()
    torch.cuda.synchronize()
    assert float(y[0]) == 1.0


def test_gate_holds_then_releases():
    from kair_amd import _hip as H
    torch.cuda.synchronize()
    H.gate_hold(5000)
    y = _axpy_burst(H, 2)
    assert H.gate_status() == 0          # still held: nothing behind the gate ran
    H.gate_release()
    torch.cuda.synchronize()
    assert H.gate_status() == 1
    assert float(y[0]) == 2.0


def test_gate_times_out():
    from kair_amd import _hip as H
    torch.cuda.synchronize()
    H.gate_hold(50)
    torch.cuda.synchronize()             # nobody releases: the wave leaves at its time limit
    assert H.gate_status() == 2
