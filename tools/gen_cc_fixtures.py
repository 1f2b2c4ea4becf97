#!/usr/bin/env python3
"""Golden vectors for the centralised-critic observation builder, from the REFERENCE's own function.

Runs only in the build container. central_critic_observer (models/CC_Model.py:196-214) is a pure
NumPy function; its module imports RLlib / torch (absent here), so this script parses the reference
file, takes that one function definition and executes it against NumPy (nothing is copied into the
repository; the outputs are data). The opponent actions are then filled in as FillInActions
(:165-193) does, np.clip(a, -1, 1) per opponent in agent order, and each agent's dict is flattened
in RLlib's order for the Dict space (sorted keys: opponent_action, opponent_obs, own_obs).

    python tools/gen_cc_fixtures.py        # -> tests/golden/cc_obs.npz
"""
import ast
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_fixtures import OUT, REF  # noqa: E402

SRC = os.path.join(REF, "models", "CC_Model.py")


def reference_observer():
    tree = ast.parse(open(SRC).read())
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "central_critic_observer"][0]
    ns = {"np": np}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), SRC, "exec"), ns)
    return ns["central_critic_observer"]


def main():
    if not os.path.isdir(REF):
        print("reference not mounted; nothing to do (fixtures are committed)")
        return
    observer = reference_observer()
    out = {}
    rs = np.random.RandomState(5)
    for name, case in (("MAIM4", "C2_MAIM4"), ("MAIM_div1", "C4_MAIM_div1"), ("MAIM8", "MAIM8_td")):
        z = np.load(os.path.join(OUT, case + ".npz"), allow_pickle=False)
        obs = z["obs"][:6, :5]                                  # [E, T, N, F] reference observations
        E, T, N, F = obs.shape
        act = rs.uniform(-1.6, 1.6, size=(E, T, N))
        act[0, 0] = [-1.0, 1.0] * (N // 2)                      # clip edges
        ids = ["agent_%d" % i for i in range(N)]
        cc = np.zeros((E, T, N, N * F + N - 1))
        for e in range(E):
            for t in range(T):
                new = observer({ids[i]: obs[e, t, i].copy() for i in range(N)})
                for i, k in enumerate(ids):
                    others = [j for j in range(N) if j != i]
                    new[k]["opponent_action"][:] = [np.clip(act[e, t, j], -1, 1) for j in others]
                    cc[e, t, i] = np.concatenate([new[k][key] for key in sorted(new[k])])
        out[name + "/obs"] = obs
        out[name + "/actions"] = act
        out[name + "/cc"] = cc
        print(name, cc.shape)
    np.savez_compressed(os.path.join(OUT, "cc_obs.npz"), **out)


if __name__ == "__main__":
    main()
