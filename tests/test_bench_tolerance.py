"""bench.py's RCCL tolerance check (order_bound_check): an fp32 SUM over n
ranks in another reduction order stays within 2 gamma_{n-1} sum_i |x_i| of
the oracle's order (BASELINE north_star: reduction-order bounded, scaled by
rank count).  Exercised here on CPU with the orders an allreduce can take --
sequential, reversed, pairwise tree, random permutations of the ranks -- on
data with heavy cancellation, and shown to reject a result off by more."""
import numpy as np
import pytest

import bench


def _order_sum(xs, order):
    acc = xs[order[0]].copy()
    for r in order[1:]:
        acc = (acc + xs[r]).astype(np.float32)
    return acc


def _tree_sum(xs):
    level = [x.copy() for x in xs]
    while len(level) > 1:
        nxt = [(level[i] + level[i + 1]).astype(np.float32) for i in range(0, len(level) - 1, 2)]
        if len(level) % 2:
            nxt.append(level[-1])
        level = nxt
    return level[0]


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_other_orders_stay_within_the_bound(n):
    rng = np.random.default_rng(n)
    m = 200_000
    # mixed magnitudes and signs: cancellation makes the relative error of a
    # result large, the bound is relative to sum |x_i|
    xs = [(rng.standard_normal(m) * 10.0 ** rng.integers(-3, 4, m)).astype(np.float32) for _ in range(n)]
    abs_sum = np.sum([np.abs(x.astype(np.float64)) for x in xs], axis=0)
    ref = _order_sum(xs, list(range(n)))
    orders = [list(range(n))[::-1], *[list(rng.permutation(n)) for _ in range(4)]]
    worst = 0.0
    for o in orders:
        ok, frac, _ = bench.order_bound_check(_order_sum(xs, o), ref, abs_sum, n)
        assert ok, (n, o, frac)
        worst = max(worst, frac)
    ok, frac, _ = bench.order_bound_check(_tree_sum(xs), ref, abs_sum, n)
    assert ok, frac
    if n > 2:
        assert worst > 0.0          # the orders do differ: the check is not vacuous


@pytest.mark.parametrize("n", [2, 8])
def test_a_wrong_result_is_rejected(n):
    rng = np.random.default_rng(100 + n)
    xs = [rng.uniform(-1, 1, 10_000).astype(np.float32) for _ in range(n)]
    abs_sum = np.sum([np.abs(x.astype(np.float64)) for x in xs], axis=0)
    ref = _order_sum(xs, list(range(n)))
    bad = ref.copy()
    k = 1234
    gamma = (n - 1) * 2.0 ** -24 / (1 - (n - 1) * 2.0 ** -24)
    bad[k] = np.float32(bad[k] + 3 * 2 * gamma * abs_sum[k])
    ok, frac, at = bench.order_bound_check(bad, ref, abs_sum, n)
    assert not ok and at == k and frac > 1.0
    # a missing rank's contribution is far outside
    ok, _, _ = bench.order_bound_check(_order_sum(xs, list(range(n - 1))), ref, abs_sum, n)
    assert not ok
    # NaN positions must agree
    nan = ref.copy()
    nan[7] = np.nan
    ok, _, at = bench.order_bound_check(nan, ref, abs_sum, n)
    assert not ok and at == 7
