"""Cost model of the model-based tuner (reference autotuning/tuner/cost_model.py
``XGBoostCostModel``: gradient-boosted trees over the numeric values of each flattened
experiment config, refit after every measurement).

XGBoost is not part of this image; scikit-learn's ``GradientBoostingRegressor`` is the same model
family (additive regression trees on squared loss). Features are generic -- every numeric leaf of
the experiment's overrides, in a fixed key order, with log2 of positive integers so batch-size
style knobs are on their natural scale -- so any tuning space works, not just micro batch x stage.
With fewer than ``min_fit`` points (or without scikit-learn) it falls back to a ridge-regularised
least-squares fit on the same features."""
import math
import numbers

import numpy as np


def flatten(d, prefix=""):
    out = {}
    for k, v in (d or {}).items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(flatten(v, key + "."))
        else:
            out[key] = v
    return out


class ConfigFeaturizer:
    def __init__(self, configs):
        keys = set()
        for c in configs:
            keys.update(k for k, v in flatten(c).items() if isinstance(v, (numbers.Number, bool)))
        self.keys = sorted(keys)

    def __call__(self, cfg):
        f = flatten(cfg)
        row = []
        for k in self.keys:
            v = f.get(k, 0)
            v = float(v) if isinstance(v, (numbers.Number, bool)) else 0.0
            row.append(math.log2(v) if v >= 1 and float(v).is_integer() else v)
        return row


class CostModel:
    """fit(X, y) / predict(X). ``kind`` 'gbt' (boosted trees, default) or 'linear'."""

    def __init__(self, kind="gbt", min_fit=4, seed=0):
        self.kind, self.min_fit, self.seed = kind, min_fit, seed
        self._model = None
        self._w = None

    def fit(self, X, y):
        X, y = np.asarray(X, dtype=np.float64), np.asarray(y, dtype=np.float64)
        self._model = None
        if self.kind == "gbt" and len(y) >= self.min_fit:
            try:
                from sklearn.ensemble import GradientBoostingRegressor
                self._model = GradientBoostingRegressor(n_estimators=64, max_depth=3, learning_rate=0.2,
                                                        random_state=self.seed).fit(X, y)
                return self
            except ImportError:  # pragma: no cover - sklearn is in the image
                pass
        Xb = np.hstack([X, np.ones((len(X), 1))])
        lam = 1e-3 * np.eye(Xb.shape[1])
        self._w = np.linalg.solve(Xb.T @ Xb + lam, Xb.T @ y)
        return self

    def predict(self, X):
        X = np.asarray(X, dtype=np.float64)
        if self._model is not None:
            return self._model.predict(X)
        return np.hstack([X, np.ones((len(X), 1))]) @ self._w
