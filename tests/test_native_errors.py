"""Legible native failures (csrc/common.hpp ATE_LAUNCH / ATE_CHECK_LAUNCH, csrc/errors.hip,
_native.call): a failed launch reaches Python as NativeError naming the HIP error, the entry
point and the launch site; an error left pending by an earlier HIP call is reported as
stale instead of as the launch's own (the round-5 "ate_forest_fit_exact failed with status
1", profiles/r05_debug/README.md). The decoding is pinned here on the CPU with a stand-in
library; tests/test_gpu.py::test_invalid_launch_is_named runs a real refused launch."""
import ctypes

import pytest

from ate_replication_causalml_amd import _native


def test_describe_status():
    assert _native.describe_status(1) == "hipErrorInvalidValue (1)"
    assert _native.describe_status(701) == "hipErrorLaunchOutOfResources (701)"
    assert _native.describe_status(12345).endswith("(12345)")
    assert "argument check" in _native.describe_status(-1)


class _Lib:
    """Stand-in for libatehip's error entry points (ctypes string buffers, int codes)."""

    def __init__(self, last=(0, b""), stale=(0, b"")):
        self.last, self.stale, self.cleared = last, stale, False

    @staticmethod
    def _fill(rec, buf, n):
        ctypes.memmove(buf, rec[1][:n - 1] + b"\0", min(len(rec[1]) + 1, n))
        return rec[0]

    def ate_last_error(self, buf, n):
        return self._fill(self.last, buf, n)

    def ate_last_stale_error(self, buf, n):
        return self._fill(self.stale, buf, n)

    def ate_clear_errors(self):
        self.cleared = True
        return 0


def test_status_detail_uses_the_native_record():
    msg = (b"hipErrorInvalidValue (1): invalid argument; kernel launch failed in "
           b"ate_forest_fit_exact at csrc/forest_exact.hip:1121")
    lib = _Lib(last=(1, msg))
    d = _native.status_detail(lib, 1)
    assert d == msg.decode() and lib.cleared
    e = _native.NativeError("ate_forest_fit_exact", 1, d)
    assert "hipErrorInvalidValue" in str(e) and "forest_exact.hip:1121" in str(e)
    assert e.entry == "ate_forest_fit_exact" and e.status == 1


def test_status_detail_stale_and_mismatch():
    stale = b"hipErrorInvalidValue (1): invalid argument; pending before a launch"
    lib = _Lib(last=(700, b"hipErrorIllegalAddress (700): ..."), stale=(1, stale))
    d = _native.status_detail(lib, 1)          # the record is another status's: decode only
    assert d.startswith("hipErrorInvalidValue (1)") and "stale" in d and stale.decode() in d
    assert _native.status_detail(_Lib(), -2).startswith("rejected by the entry point")


def test_call_raises_named_error(monkeypatch):
    class Lib(_Lib):
        def ate_fake(self, *a):
            return 9
    lib = Lib(last=(9, b"hipErrorInvalidConfiguration (9): bad block; kernel launch failed "
                       b"in ate_fake at csrc/x.hip:1"))
    monkeypatch.setattr(_native, "hip", lambda: lib)
    with pytest.raises(_native.NativeError, match=r"ate_fake failed with status 9: "
                                                   r"hipErrorInvalidConfiguration"):
        _native.call("ate_fake")
