"""MI355X-native average-treatment-effect framework (gfx950 HIP kernels + RCCL).

Capability parity with the R replication of Athey & Imbens' causal-ML ATE tutorial
(ate_functions.R + ate_replication.Rmd): 14 estimators, the synthetic/real data
pipeline, and the large-N K-fold DML cross-fit. See ``api`` for the entry points.
"""
import os as _os

# Hardware queues per process (HIP's default is 4). Independent launches on separate HIP
# streams -- the 3K forests of a cross-fit, the fits in flight of bench.py -- share that
# many queues, so with 4 at most 4 forest launches ran at once: the per-GPU shard of
# BASELINE config 3 (15 forests of 13 trees) kept 52 of 256 CUs busy, 77 s -> 35 s with 16
# (profiles/r02c_gram/cfg3_hwq.log; the headline step is unchanged). HIP reads it when
# its library loads, so it applies when this package is imported before torch; a lower
# inherited value (the MI355X boxes export HIP's default, 4) is raised to 16.
# ATE_HW_QUEUES=<n> picks another value, ATE_HW_QUEUES=0 leaves the environment alone.
# The change is logged (logger "ate_replication_causalml_amd", INFO) and recorded in
# ``HW_QUEUES`` = (inherited, set, effective); when HIP was already initialised in this
# process (a GPU call before this import) the new value cannot take effect: a warning says so.
import logging as _logging
import sys as _sys

_log = _logging.getLogger(__name__)
_want = min(int(_os.environ.get("ATE_HW_QUEUES", "16")), 32)
_old = _os.environ.get("GPU_MAX_HW_QUEUES")
HW_QUEUES = (_old, _old, True)
if _want > 0 and int(_old or 0) < _want:
    _torch = _sys.modules.get("torch")
    _late = bool(_torch is not None and getattr(_torch, "cuda", None) is not None
                 and _torch.cuda.is_initialized())
    _os.environ["GPU_MAX_HW_QUEUES"] = str(_want)
    HW_QUEUES = (_old, str(_want), not _late)
    _log.info("GPU_MAX_HW_QUEUES %s -> %d (set ATE_HW_QUEUES=0 to leave it alone)", _old, _want)
    if _late:
        import warnings as _warnings
        _warnings.warn(f"GPU_MAX_HW_QUEUES raised to {_want} after HIP was initialised: it has "
                       "no effect in this process (import ate_replication_causalml_amd before "
                       "any GPU call)", RuntimeWarning, stacklevel=2)
from .api import (Replication, ate_aipw_crossfit, ate_aipw_glm, ate_aipw_rf, ate_belloni, ate_causal_forest,
                  ate_causal_forest_bootstrap,
                  ate_dml, ate_double_ml, ate_ipw, ate_ipw_wls, ate_lasso, ate_lasso_single,
                  ate_naive, ate_ols, ate_residual_balance, propensity_lasso,
                  propensity_logistic, replicate)
from .config import BalanceConfig, CvConfig, ForestConfig, ReplicateConfig, RunConfig
from .result import AteResult, format_table, results_frame

__version__ = "0.1.0"
