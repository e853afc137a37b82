"""Reference (T-ref) forests: the host C++ engine (csrc/cpu/forest_cpu.cpp) behind the
randomForest / grf semantics of SURVEY.md N5/N6 (see models/forest.py). The GPU kernels
grow bit-identical trees, so this is also the parity oracle for csrc/forest.hip."""
from ..models.forest import (average_treatment_effect, causal_forest, fit_forest,  # noqa: F401
                             regression_forest, rf_classifier)


def rf_classifier_fit(X, y, num_trees=500, seed=1, mtry=None, nodesize=1, splits="binned"):
    return rf_classifier(X, y, num_trees=num_trees, mtry=mtry, nodesize=nodesize, seed=seed,
                         backend="cpu", splits=splits)
