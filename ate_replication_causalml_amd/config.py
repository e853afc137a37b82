"""Typed configuration.

The reference configures through function defaults (``num_trees=100``,
``bootstrap_se=F``, ``optimizer="quadprog"``; ate_functions.R:3-393) and hard-coded
driver constants (n_obs=50000, seed 1991, pt=pc=0.85, 2500/2000/2000 trees;
ate_replication.Rmd:42-43,99-100,217,232,253). Every default below equals the
reference's value at its call site in the driver.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field, replace


@dataclass(frozen=True)
class RunConfig:
    backend: str = "auto"       # "gpu" | "cpu" (device path on host tensors) | "reference" (fp64 T-ref)
    dtype: str = "f64"          # panel storage for GLM/LASSO fits: f64 | f32 | bf16
    compat: str = "reference"   # reproduce reference quirks (Appendix A) or "textbook"
    seed: int = 1991            # set.seed(1991) (ate_replication.Rmd:42)

    def device(self):
        import torch
        if self.backend == "gpu":
            return torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_initialized()
                                else 0)
        if self.backend == "cpu":
            return torch.device("cpu")
        if self.backend == "auto":
            return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        return None             # reference


@dataclass(frozen=True)
class CvConfig:
    nfolds: int = 10            # cv.glmnet default
    alpha: float = 1.0
    nlambda: int = 100
    lambda_min_ratio: float | None = None
    thresh: float = 1e-7


@dataclass(frozen=True)
class ForestConfig:
    num_trees: int = 100        # doubly_robust / double_ml default (ate_functions.R:149,372)
    mtry: int | None = None     # floor(sqrt(p)) for randomForest; grf: min(ceil(sqrt(p)+20), p)
    min_node: int = 1
    seed: int = 12325


@dataclass(frozen=True)
class BalanceConfig:
    zeta: float = 0.5           # balanceHD defaults (residualBalance.ate)
    alpha: float = 0.9
    allow_negative_weights: bool = False
    scale_x: bool = True


@dataclass(frozen=True)
class ReplicateConfig:
    """The driver ate_replication.Rmd end to end (14 result rows)."""
    n_obs: int = 50_000
    pt: float = 0.85
    pc: float = 0.85
    selection_compat: str = "reference"
    dr_trees: int = 2500        # ate_replication.Rmd:217
    dml_trees: int = 2000       # :232 (num_tree= partial-matches num_trees)
    cf_trees: int = 2000        # :253
    cf_seed: int = 12345        # :255
    bootstrap_se: bool = False
    B: int = 1000
    include: tuple | None = None   # subset of method labels (None = all 14)
    run: RunConfig = field(default_factory=RunConfig)
    balance: BalanceConfig = field(default_factory=BalanceConfig)

    def to_dict(self):
        return asdict(self)

    def with_(self, **kw):
        return replace(self, **kw)


METHODS = (
    "oracle", "naive", "Direct Method", "Propensity_Weighting", "Propensity_Regression",
    "Propensity_Weighting_LASSOPS", "Single-equation LASSO", "Usual LASSO",
    "Doubly Robust with Random Forest PS", "Doubly Robust with logistic regression PS",
    "Belloni et.al", "Double Machine Learning", "residual_balancing", "Causal Forest(GRF)",
)
