"""The oracle's SURVEY §8(d) robustness RHS (std::mt19937_64 seed 12345, uniform [-1, 1),
boundary 0) against libstdc++ itself: tests/golden/mt_rhs.json comes from
tests/golden/make_mt_rhs.cpp (std::mt19937_64 + std::uniform_real_distribution)."""
import json
import pathlib

import numpy as np
import pytest

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden" / "mt_rhs.json"


@pytest.fixture(scope="module")
def fixture():
    return json.loads(GOLDEN.read_text())


def test_engine_is_the_standards_mt19937_64(oracle_mod, fixture):
    # [rand.predef]: the 10000th output of a default-constructed mt19937_64
    assert oracle_mod.lib().orc_mt64_nth(5489, 10000) == 9981545732273789042
    assert fixture["kat_default_seed_10000th"] == "9981545732273789042"


@pytest.mark.parametrize("i", [0, 1, 2])
def test_rhs_bitwise_libstdcxx(oracle_mod, fixture, i):
    case = fixture["fields"][i]
    f = oracle_mod.rhs_mt64(case["N"], case["seed"])
    assert oracle_mod.fnv_hash(f) == case["hash"]
    assert f[1, 1:5].tolist() == case["first_interior"]
    assert np.all(f[0] == 0) and np.all(f[:, -1] == 0)
    assert f.min() >= -1.0 and f.max() < 1.0
