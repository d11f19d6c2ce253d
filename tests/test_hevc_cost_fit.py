"""tools/hevc_cost_fit.py: the slice-layout simulation matches the planner's rule and the best
contiguous partition is a lower bound (synthetic unit tables; the real ones come from a GPU run)."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
import hevc_cost_fit as F  # noqa: E402


def _table(units_w=8, rows=8, seed=1):
    rng = np.random.default_rng(seed)
    n = units_w * rows
    typ = rng.integers(0, 3, n)
    cbf = (rng.random(n) < 0.4).astype(int)
    lsum = rng.integers(1, 200, n) * cbf
    sb = rng.integers(1, 10, n) * cbf
    eb = rng.integers(1, 60, n) * cbf
    tok = np.where(cbf == 0, 1, lsum // 4 + 13 * sb + 4 * eb)
    return np.stack([typ, cbf, lsum, sb, eb, tok], 1).astype(np.float64)


def test_slices_cover_every_ctb_and_respect_the_bound():
    t = _table()
    per, ct = F.slices(t, F.model_current, 8, max_slices=6, cost_per_slice=1)
    assert per.sum() == ct.sum() == t[:, 5].sum()
    assert 1 <= len(per) <= 6
    assert F.best_partition(ct, len(per)) <= per.max() + 1


def test_exact_model_balances_better_than_a_constant_one():
    t = _table(16, 16, seed=3)
    exact = lambda typ, cbf, lsum, sb, eb: np.where(cbf == 0, 1, lsum // 4 + 13 * sb + 4 * eb)  # noqa: E731
    flat = lambda typ, cbf, lsum, sb, eb: np.ones_like(cbf, dtype=np.float64)  # noqa: E731
    best, _ = F.slices(t, exact, 16, max_slices=8, cost_per_slice=1)
    naive, _ = F.slices(t, flat, 16, max_slices=8, cost_per_slice=1)
    assert best.max() <= naive.max()
