"""CommWatchdog logic on the CPU (the RCCL-side behaviour runs on the GPU in
tests/test_gpu_rccl.py::test_rccl_watchdog_*): completion events are
stand-in objects with a query() method, so the timeout, the guarded wait and
the asynchronous raise in the main thread are exercised without a device.
Reference: the reference's MPI path has no failure handling at all
(OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:289-297); SURVEY §5.3."""
import time

import pytest

from gelim.parallel import comm as C


class _Ev:
    def __init__(self, done_at=None):
        self.done_at = done_at

    def query(self):
        return self.done_at is not None and time.monotonic() >= self.done_at


def _wd(timeout_s):
    return C.CommWatchdog(timeout_s=timeout_s, poll_s=0.01)


def test_wait_event_completes():
    wd = _wd(2.0)
    try:
        wd.wait_event(_Ev(time.monotonic() + 0.05), "test")
        assert wd.error is None
    finally:
        wd.stop()


def test_wait_event_times_out():
    wd = _wd(0.2)
    try:
        t0 = time.monotonic()
        with pytest.raises(C.CommFailure, match="peer rank died or hung"):
            wd.wait_event(_Ev(None), "stuck collective")
        assert 0.15 <= time.monotonic() - t0 < 1.5
        with pytest.raises(C.CommFailure):  # sticky: every later wait raises too
            wd.wait_event(_Ev(time.monotonic()), "later")
    finally:
        wd.stop()


def test_tracked_event_raises_in_main_thread():
    wd = _wd(0.2)
    try:
        wd.track(_Ev(None), "broadcast")
        t0 = time.monotonic()
        with pytest.raises(C.CommFailure):
            for _ in range(300):
                time.sleep(0.01)
        assert time.monotonic() - t0 < 2.0
        assert wd.error is not None
    finally:
        wd.stop()


def test_completed_events_are_dropped():
    wd = _wd(0.3)
    try:
        now = time.monotonic()
        for k in range(5):
            wd.track(_Ev(now + 0.01 * k), f"c{k}")
        time.sleep(0.6)
        assert wd.error is None and not wd._pending
    finally:
        wd.stop()


def test_paused_during_capture():
    """While a capture is in progress nothing is queried or timed out, and
    the ages restart when it ends."""
    wd = _wd(0.15)
    try:
        with wd.paused():
            wd.track(_Ev(time.monotonic() + 0.5), "captured")
            time.sleep(0.4)
            assert wd.error is None
        time.sleep(0.05)
        assert wd.error is None
        time.sleep(0.3)  # done at +0.5 s: completed before its restarted age passes the timeout
        assert wd.error is None
    finally:
        wd.stop()
