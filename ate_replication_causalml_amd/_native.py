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


c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_uint64 = ctypes.c_uint64
c_double = ctypes.c_double

# name -> argtypes (restype int). 'p' pointer, 'i' int32, 'l' int64, 'u' uint64, 'd' double
_SIGS = {
    "ate_gram_bf16": "pliipipipipppp",
    "ate_gram_bf16_pair": "pllipippipippipp",
    "ate_gram_bf16_tri": "pllippipippipp",
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
    "ate_dgp_fill": "iplllllp" + "uiipp",
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


def hip():
    """The gfx950 kernel library; raises NativeMissing if it was not built."""
    global _hip
    if _hip is None:
        import torch  # noqa: F401  (ensure torch's HIP runtime is loaded first)
        # ATE_HIP_LIB: an alternative build of the same library (e.g. the cycle-profiling
        # variant made by tools/enet_profile.py); ATE_DEBUG=1: the device-assertion build
        # (_build.py, csrc/common.hpp ATE_DASSERT)
        debug = os.environ.get("ATE_DEBUG", "0") not in ("", "0")
        p = Path(os.environ["ATE_HIP_LIB"]) if os.environ.get("ATE_HIP_LIB") else \
            _LIBDIR / ("libatehip_debug.so" if debug else "libatehip.so")
        if not p.exists():
            raise NativeMissing(
                f"{p} not found: build it with `python -m ate_replication_causalml_amd._build` "
                "(hipcc --offload-arch=gfx950). GPU ops have no fallback.")
        _hip = _load(p, _SIGS)
    return _hip


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
    """Invoke a kernel-library entry point and raise on a non-zero status."""
    f = getattr(hip(), name)
    rc = f(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")
    return rc


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
