"""The lane-level restatement of k_als_wave (tests/als_wave_model.py) solves
the ALS normal equations: checked against np.linalg.solve on the augmented
system [Z, 1] (CPU, float64, so the bar is rounding-level).  Covers one, two
and four 32-wide tile rows, padding columns (k < 32 NT), fewer ratings than
rows, and a rank-deficient Gramian made regular only by reg."""

import numpy as np
import pytest

from als_wave_model import solve


@pytest.mark.parametrize("nt,k,n", [(1, 20, 90), (1, 32, 7), (2, 64, 90), (2, 48, 30),
                                    (4, 100, 90), (4, 128, 200)])
def test_wave_model_solves_normal_equations(nt, k, n):
    rs = np.random.RandomState(nt * 1000 + k + n)
    Z = rs.normal(0, 0.3, (n, k))
    t = rs.normal(0, 1, n)
    reg = 0.1
    Y = np.hstack([Z, np.ones((n, 1))])
    x = np.linalg.solve(Y.T @ Y + reg * np.eye(k + 1), Y.T @ t)
    w, b = solve(nt, k, Z, t, reg)
    scale = max(1.0, np.abs(x).max())
    assert np.abs(w - x[:k]).max() <= 1e-9 * scale
    assert abs(b - x[k]) <= 1e-9 * scale
