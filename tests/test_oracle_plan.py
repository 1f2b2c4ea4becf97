"""Pin the plan-replay restatement (oracle/plan.py) against the reference's own outputs.

tests/golden/plan_replay.npz was produced by running the LP scripts' evaluation loop
(SHLP_8.py:737-766) on the reference env classes with LP-like plans (tools/gen_plan_fixtures.py).
Every comparison is exact: per-step rewards and episode returns float64-bit-equal, the
observation sums integer-equal.
"""
import numpy as np
import pytest

from golden_io import load_base_stock
from oracle import plan as pl

META, CASES = load_base_stock("plan_replay.npz")


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_plan_replay_matches_reference(name):
    m, d = META[name], CASES[name]
    out = pl.plan_rollout(m["kind"], m["config"], d["plans"], per_episode=m["layout"] == "episode",
                          demand=d["demand"])
    np.testing.assert_array_equal(out["rewards"], d["rewards"])
    np.testing.assert_array_equal(out["return"], d["return"])
    for k in ("inventory", "backlog", "customer_backlog"):
        np.testing.assert_array_equal(out[k], d[k])
