"""The fp32-Gram CV path kernel (csrc/enet.hip enet_path_kernel<float, LASSO>) against the
float64 CPU reference of the same cv.glmnet problems (reference/glmnet.py semantics).

The bench's bf16/f32 panels run the fp32 instantiation: small active sets in mode S (one wave
over all p coordinates, the moved coordinates' Gram columns cached in LDS), then mode L
(64-coordinate blocks with helper-wave pulls). These cases cover both regimes and the switch
between them, p not a multiple of 64, an unpenalised coordinate, the lasso and the
elastic-net instantiations, and the nested cross-fit sets (fold problems consuming their full
problem's lambdas). Tolerances are those of an fp32 Gram (rel ~1e-7 per entry)."""
import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.ops import gram as gram_op
from ate_replication_causalml_amd.ops.enet import cv_enet_gaussian
from ate_replication_causalml_amd.ops.panel import build_panel
from ate_replication_causalml_amd.parallel import rng

pytestmark = pytest.mark.gpu


def _problem(n, p, k_signal, seed, corr=0.0):
    rs = np.random.RandomState(seed)
    f = rs.randn(n, 1)
    X = rs.randn(n, p) + corr * f
    beta = np.zeros(p)
    beta[:k_signal] = rs.choice([-1.0, 1.0], k_signal) * rs.uniform(0.2, 1.0, k_signal)
    y = X @ beta + rs.randn(n)
    return X, y


def _compare(gpu, X, y, alpha, pf=None, full_sets=None, nfolds=5, atol=2e-5):
    n = len(y)
    fid = rng.fold_ids(n, nfolds, 1)
    pan = build_panel(X, None, y, folds=fid, dtype="f32", device=gpu)
    G = gram_op.gram(pan)
    kw = dict(penalty_factor=pf, alpha=alpha, full_sets=full_sets)
    rg = cv_enet_gaussian(G, pan, pan.xcols, [pan.cols["Y"]], **kw)
    rc = cv_enet_gaussian(G.cpu(), pan, pan.xcols, [pan.cols["Y"]], **kw)
    rg.check()
    nf = rc.nlam.shape[0]
    for f in range(nf):
        nl = int(rc.nlam[f])
        assert abs(int(rg.nlam[f]) - nl) <= 1
        nl = min(nl, int(rg.nlam[f]))
        # same lambda sequence (computed from the same fp32 Gram on both sides)
        np.testing.assert_allclose(rg.lambdas[f, :nl].cpu().numpy(), rc.lambdas[f, :nl].numpy(),
                                   rtol=1e-6)
        # coefficient paths agree to the fp32 C the kernel walks on (the reference walks the
        # fp64 standardisation of the same Gram)
        scale = np.abs(rc.coef_path[f, :nl].numpy()).max() + 1.0
        np.testing.assert_allclose(rg.coef_path[f, :nl].cpu().numpy(),
                                   rc.coef_path[f, :nl].numpy(), atol=atol * scale)
        np.testing.assert_allclose(rg.cvm[f, :nl].cpu().numpy(), rc.cvm[f, :nl].numpy(),
                                   rtol=1e-4)
    return rg, rc


@pytest.mark.parametrize("alpha", [1.0, 0.5])
def test_fp32_path_small_active_set(gpu, alpha):
    """p = 70 (two blocks, the second partial), 4 signals: the active set stays small, so
    the whole path runs in mode S; an unpenalised last coordinate enters at lambda_max."""
    X, y = _problem(4000, 70, 4, 11)
    pf = np.ones(70)
    pf[-1] = 0.0
    _compare(gpu, X, y, alpha, pf=pf)


@pytest.mark.parametrize("alpha", [1.0, 0.7])
def test_fp32_path_mode_switch(gpu, alpha):
    """p = 300, 120 correlated signals: more than ENET_S_ENTER coordinates move early, so the
    problem leaves mode S for the blocked walk part-way along the path."""
    X, y = _problem(6000, 300, 120, 12, corr=0.5)
    _compare(gpu, X, y, alpha, atol=5e-5)


def test_fp32_path_nested_crossfit_sets(gpu):
    """The DML nuisance layout: K full training sets (all segments but k), each with its own
    K-1 fold problems that consume the full problem's lambda sequence as it is published."""
    X, y = _problem(5000, 130, 10, 13, corr=0.3)
    K = 5
    full_sets = [[s for s in range(K) if s != k] for k in range(K)]
    rg, rc = _compare(gpu, X, y, 1.0, full_sets=full_sets, nfolds=K)
    assert torch.equal(rg.sel.cpu().long(), rc.sel.long())
