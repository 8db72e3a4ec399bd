"""Cost model of the model-based tuner (reference autotuning/tuner/cost_model.py ``XGBoostCostModel``: xgboost is
not part of this stack, so the same role is played by scikit-learn's gradient-boosted trees, with a least-squares
fallback when scikit-learn is missing)."""
import numpy as np


class CostModel:

    def __init__(self, loss_type="reg", seed=0):
        self.loss_type = loss_type
        self.seed = seed
        self.model = None
        self._lsq = None

    def fit(self, xs, ys):
        xs = np.asarray(xs, dtype=np.float64)
        ys = np.asarray(ys, dtype=np.float64)
        if self.loss_type == "rank" and ys.size:
            ys = ys.argsort().argsort().astype(np.float64)  # fit the ranks: only the ordering matters
        try:
            from sklearn.ensemble import GradientBoostingRegressor
            self.model = GradientBoostingRegressor(n_estimators=min(200, 20 * max(len(ys), 1)), max_depth=3,
                                                   learning_rate=0.1, random_state=self.seed)
            self.model.fit(xs, ys)
        except ImportError:
            a = np.hstack([xs, np.ones((len(xs), 1))])
            self._lsq, *_ = np.linalg.lstsq(a, ys, rcond=None)

    def predict(self, xs):
        xs = np.asarray(xs, dtype=np.float64)
        if self.model is not None:
            return self.model.predict(xs)
        if self._lsq is not None:
            return np.hstack([xs, np.ones((len(xs), 1))]) @ self._lsq
        return np.zeros(len(xs))
