"""GPU: coarse levels entered with x0 = 0 do not store the pre-smoothed iterate; k_post
recomputes it from f (x1 = J(0), x2 = J(x1), or x1 when the pre-smoothing check fired).
Bit-identical to the reference in every early-exit combination (eps sweep on a random
problem so the pre and post checks of the coarse levels fire in turn), V and W cycles,
and equal to the stored-iterate path (PGMG_FLAG_NO_RECOMPUTE)."""
import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _problem(N, seed):
    rng = np.random.default_rng(seed)
    phi0 = rng.uniform(-1, 1, (N, N))
    f = rng.uniform(-1, 1, (N, N)) * 1e-3
    for a in (phi0, f):
        a[0, :] = a[-1, :] = a[:, 0] = a[:, -1] = 0.0
    return phi0, f


@pytest.mark.parametrize("kind", ["V", "W"])
def test_recompute_eps_sweep_matches_oracle(pgmg, oracle_mod, kind, monkeypatch):
    N = 129
    phi0, f = _problem(N, 5)
    exits_seen = 0
    for eps in [10 ** (k / 6.0) for k in range(30, -12, -1)]:
        o = oracle_mod.Oracle(eps=eps)
        ref = phi0.copy()
        for _ in range(3):
            (o.v_cycle if kind == "V" else o.w_cycle)(ref, f)
        exits_seen += o.early_exits
        for rec in ("1", "0"):
            fl = pgmg.PGMG_FLAG_NO_CROSS | (pgmg.PGMG_FLAG_NO_RECOMPUTE if rec == "0" else 0)
            with pgmg.Solver(N, eps=eps, tail_n=9, flags=fl) as s:
                s.set_problem(phi0, f)
                (s.vcycle if kind == "V" else s.wcycle)(3)
                assert_bitwise(s.solution(), ref, f"{kind} eps={eps} recompute={rec}")
                assert s.stats()[0] == o.sweeps, (kind, eps, rec)
    assert exits_seen > 0


def test_recompute_bytes_accounting(pgmg, monkeypatch):
    """pgmg_vcycle_bytes drops the stored iterate of the coarse levels (16 B/point)."""
    N = 1025
    b = {}
    for rec in ("1", "0"):
        fl = pgmg.PGMG_FLAG_NO_CROSS | (pgmg.PGMG_FLAG_NO_RECOMPUTE if rec == "0" else 0)
        with pgmg.Solver(N, flags=fl) as s:
            b[rec] = s.vcycle_bytes()
    n1 = (513 - 2) ** 2
    assert b["0"] - b["1"] > 16 * n1
