"""ctypes bindings of the in-tree native libraries.

``hip()`` returns the gfx950 kernel library (``_lib/libatehip.so``). It is loaded
lazily, after ``import torch`` (torch's HIP runtime is the one the process uses;
both share the ``libamdhip64.so.7`` soname). If the library is missing while a GPU
op is requested, :class:`NativeMissing` is raised — there is no silent fallback.
``cpu()`` returns the host C++ library (forest engine).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_LIBDIR = Path(__file__).resolve().parent / "_lib"
_hip = None
_cpu = None


class NativeMissing(RuntimeError):
    pass


class NativeError(RuntimeError):
    """A kernel-library entry point returned a non-zero status. ``status``: the HIP error
    code (> 0, named in the message with its entry point, file and line) or the entry
    point's own argument check (< 0)."""

    def __init__(self, name: str, status: int, detail: str):
        self.entry, self.status = name, status
        super().__init__(f"{name} failed with status {status}: {detail}")


# hip_runtime_api.h hipError_t (ROCm 7.2), for statuses whose native message is unavailable
HIP_ERRORS = {
    1: "hipErrorInvalidValue", 2: "hipErrorOutOfMemory", 3: "hipErrorNotInitialized",
    4: "hipErrorDeinitialized", 9: "hipErrorInvalidConfiguration",
    13: "hipErrorInvalidSymbol", 17: "hipErrorInvalidDevicePointer",
    21: "hipErrorInvalidMemcpyDirection", 35: "hipErrorInsufficientDriver",
    52: "hipErrorMissingConfiguration", 53: "hipErrorPriorLaunchFailure",
    98: "hipErrorInvalidDeviceFunction", 100: "hipErrorNoDevice", 101: "hipErrorInvalidDevice",
    200: "hipErrorInvalidImage", 201: "hipErrorInvalidContext", 209: "hipErrorNoBinaryForGpu",
    218: "hipErrorInvalidKernelFile", 400: "hipErrorInvalidHandle", 500: "hipErrorNotFound",
    600: "hipErrorNotReady", 700: "hipErrorIllegalAddress", 701: "hipErrorLaunchOutOfResources",
    702: "hipErrorLaunchTimeOut", 710: "hipErrorAssert", 719: "hipErrorLaunchFailure",
    720: "hipErrorCooperativeLaunchTooLarge", 801: "hipErrorNotSupported",
    900: "hipErrorStreamCaptureUnsupported", 901: "hipErrorStreamCaptureInvalidated",
    907: "hipErrorCapturedEvent", 999: "hipErrorUnknown",
}


def describe_status(rc: int) -> str:
    """Name of an entry point's non-zero status without the library's message."""
    if rc < 0:
        return "rejected by the entry point's own argument check (no kernel launched)"
    return f"{HIP_ERRORS.get(rc, 'hipError?')} ({rc})"


c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_uint64 = ctypes.c_uint64
c_double = ctypes.c_double

# name -> argtypes (restype int). 'p' pointer, 'i' int32, 'l' int64, 'u' uint64, 'd' double
_SIGS = {
    "ate_gram_bf16": "pliipipipipppp",
    "ate_gram_bf16_pair": "pllipippipippippp",
    "ate_gram_bf16_tri": "pllippipippipp",
    "ate_gram_pair_bal": "",
    "ate_last_error": "pi",
    "ate_last_stale_error": "pi",
    "ate_clear_errors": "",
    "ate_debug_bad_launch": "ip",
    "ate_check_kernel_resources": "pi",
    "ate_gram_f32": "plippipipippppp",
    "ate_gram_f64": "plippipipippppp",
    "ate_gram_tile_sizes": "pppp",
    "ate_chol_solve": "pipiipdpppppp",
    "ate_chol_solve_k": "pipipidppppp",
    "ate_spd_solve_batched": "ppiippp",
    "ate_predict": "ipllppiidipp",
    "ate_irls_update": "ipllppiiiiippppipp",
    "ate_irls_check": "piidippp",
    "ate_naive": "ippplpppp",
    "ate_clip_propensity": "pplpp",
    "ate_aipw": "ppppppldpppp",
    "ate_dml_moments": "ppplppp",
    "ate_dml_finalize": "pipp",
    "ate_boot_multinomial": "ppluiipp",
    "ate_boot_poisson": "ppluiilipp",
    "ate_enet_isa_selftest": "pp",
    "ate_enet_prepare": "piipipiipipipppppppp",
    "ate_enet_path": "pipiippppidddipppppippp",
    "ate_enet_coef": "ppiiiipppppppp",
    "ate_enet_cvloss_gauss": "pippiipppiiipp",
    "ate_cv_select": "pppiipippppip",
    "ate_enet_pick": "ppiiipppip",
    "ate_dml_resid_moments": "ipllpipipiiiiiippp",
    "ate_dml_resid_exact": "pllpipipiiiiiiippp",
    "ate_lognet_path": "iplpiipipipdddippippppppppp",
    "ate_lognet_cvloss": "iplpiippipppipp",
    "ate_dgp_fill": "iplllllp" + "uiipppp",
    "ate_sel_block_rows": "",
    "ate_sel_gen_count": "upilllpp",
    "ate_sel_gen_flags": "upillpp",
    "ate_sel_gen_mark": "upiplllpiplp",
    "ate_forest_fit": "pppppi" + "pppppppp" + "ip",
    "ate_forest_predict": "ppiiipppppippip",
    "ate_forest_pack": "pippppppp",
    "ate_forest_scratch_bytes": "ii",
    "ate_forest_exact_scratch_bytes": "iiii",
    "ate_forest_fit_exact": "piiipppippppippppppppp",
    "ate_forest_predict16": "ppiiipppppppippip",
    "ate_bin_matrix": "plipppp",
    "ate_panel_xtv": "iplpipplipp",
    "ate_select_compact": "plppddpppp" + "p",
    "ate_gbdt_run": "ppp",
    "ate_lv_boot": "ppp",
    "ate_lv_classify": "pipiippp",
    "ate_lv_decide": "ppipipipippppp" + "iipip",
    "ate_lv_partition": "ppipippppipp",
    "ate_lv_scatter": "pppppippp",
    "ate_lv_children": "pippppp",
    "ate_lv_transpose": "piipip",
    "ate_gbdt_bin_panel": "pilpipppilpppl" + "p",
    "ate_gbdt_slab_entries": "liii",
    "ate_gbdt_slab2_entries": "li",
    "ate_gbdt_pair_root": "pppplllp",
    "ate_gbdt_apply": "plliipppp" + "p",
    "ate_panel_xv": "iplpipiplpp",
    "ate_col_moments": "pllipppp",
    "ate_standardize": "pllippp",
    "ate_interactions": "pllipl" + "p",
    "ate_scan_parts": "l",
    "ate_gbdt_limits": "p",
    "ate_excl_scan_i32": "plpppp",
    "ate_excl_scan_i64": "plpppp",
}
_RESTYPE = {"ate_forest_scratch_bytes": ctypes.c_int64,
            "ate_forest_exact_scratch_bytes": ctypes.c_int64, "ate_gbdt_slab_entries": ctypes.c_int64,
            "ate_gbdt_slab2_entries": ctypes.c_int64,
            "ate_scan_parts": ctypes.c_int64}
_CT = {"p": c_void_p, "i": c_int, "l": c_int64, "u": c_uint64, "d": c_double}


def _load(path: Path, sigs: dict):
    lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
    for name, sig in sigs.items():
        if hasattr(lib, name):
            f = getattr(lib, name)
            f.restype = _RESTYPE.get(name, c_int)
            f.argtypes = [_CT[ch] for ch in sig]
    return lib


def hip_available() -> bool:
    return (_LIBDIR / "libatehip.so").exists()


def hip_library_path() -> Path:
    """The kernel library hip() loads: ATE_HIP_LIB, else the debug build under ATE_DEBUG=1,
    else _lib/libatehip.so."""
    debug = os.environ.get("ATE_DEBUG", "0") not in ("", "0")
    return Path(os.environ["ATE_HIP_LIB"]) if os.environ.get("ATE_HIP_LIB") else \
        _LIBDIR / ("libatehip_debug.so" if debug else "libatehip.so")


def hip():
    """The gfx950 kernel library; raises NativeMissing if it was not built."""
    global _hip
    if _hip is None:
        import torch  # noqa: F401  (ensure torch's HIP runtime is loaded first)
        # ATE_HIP_LIB: an alternative build of the same library (e.g. the cycle-profiling
        # variant made by tools/enet_profile.py); ATE_DEBUG=1: the device-assertion build
        # (_build.py, csrc/common.hpp ATE_DASSERT)
        debug = os.environ.get("ATE_DEBUG", "0") not in ("", "0")
        p = hip_library_path()
        if not p.exists():
            raise NativeMissing(
                f"{p} not found: build it with `python -m ate_replication_causalml_amd._build` "
                "(hipcc --offload-arch=gfx950). GPU ops have no fallback.")
        _hip = _load(p, _SIGS)
        if debug:
            _check_kernel_resources(_hip)
    return _hip


_resource_report = None


def _check_kernel_resources(lib):
    """Debug build: every registered heavy kernel's compiled attributes (max block size,
    static LDS, registers, scratch) against its launch shape, once at load
    (csrc/errors.hip ate_check_kernel_resources); a kernel that cannot launch as registered
    raises here, naming it, instead of failing later with a bare status."""
    global _resource_report
    buf = ctypes.create_string_buffer(1 << 14)
    bad = lib.ate_check_kernel_resources(buf, len(buf))
    _resource_report = buf.value.decode(errors="replace")
    if bad > 0:
        raise NativeError("ate_check_kernel_resources", bad,
                          "kernels that cannot launch as registered:\n" + "\n".join(
                              l for l in _resource_report.splitlines() if "FAIL" in l))


def kernel_resource_report() -> str | None:
    """The debug build's load-time resource check, one line per kernel (None otherwise)."""
    return _resource_report


def _native_message(lib, fn: str) -> tuple[int, str]:
    buf = ctypes.create_string_buffer(512)
    code = getattr(lib, fn)(buf, len(buf))
    return code, buf.value.decode(errors="replace")


def cpu():
    global _cpu
    if _cpu is None:
        p = _LIBDIR / "libatecpu.so"
        if not p.exists():
            from ._build import build_cpu
            build_cpu()
        _cpu = _load(p, {})
    return _cpu


def check(rc: int, name: str = "native call"):
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


def call(name: str, *args):
    """Invoke a kernel-library entry point and raise :class:`NativeError` on a non-zero
    status, with the HIP error's name and description, and the entry point, file and line
    of the failed launch (csrc/common.hpp ATE_LAUNCH / ATE_CHECK_LAUNCH). An error that was
    already pending from an earlier HIP call is reported separately, as stale."""
    lib = hip()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise NativeError(name, rc, status_detail(lib, rc))
    return rc


def status_detail(lib, rc: int) -> str:
    """The library's record of a failed launch (when it is this status's), else the decoded
    status; plus any stale error found pending before a launch."""
    detail = describe_status(rc)
    if rc > 0 and hasattr(lib, "ate_last_error"):
        code, msg = _native_message(lib, "ate_last_error")
        if code == rc and msg:
            detail = msg
        scode, smsg = _native_message(lib, "ate_last_stale_error")
        if scode and smsg:
            detail += f" [stale, cleared before the launch: {smsg}]"
        lib.ate_clear_errors()
    return detail


def loaded_libraries():
    """Paths of in-tree native libraries mapped into this process (diagnostics)."""
    out = []
    try:
        with open(f"/proc/{os.getpid()}/maps") as f:
            for line in f:
                if str(_LIBDIR) in line:
                    out.append(line.split()[-1])
    except OSError:
        pass
    return sorted(set(out))
