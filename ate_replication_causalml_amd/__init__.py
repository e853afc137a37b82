"""MI355X-native average-treatment-effect framework (gfx950 HIP kernels + RCCL).

Capability parity with the R replication of Athey & Imbens' causal-ML ATE tutorial
(ate_functions.R + ate_replication.Rmd): 14 estimators, the synthetic/real data
pipeline, and the large-N K-fold DML cross-fit. See ``api`` for the entry points.
"""
from .api import (Replication, ate_aipw_crossfit, ate_aipw_glm, ate_aipw_rf, ate_belloni, ate_causal_forest,
                  ate_causal_forest_bootstrap,
                  ate_dml, ate_double_ml, ate_ipw, ate_ipw_wls, ate_lasso, ate_lasso_single,
                  ate_naive, ate_ols, ate_residual_balance, propensity_lasso,
                  propensity_logistic, replicate)
from .config import BalanceConfig, CvConfig, ForestConfig, ReplicateConfig, RunConfig
from .result import AteResult, format_table, results_frame

__version__ = "0.1.0"
