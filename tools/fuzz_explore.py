#!/usr/bin/env python3
"""Exploratory differential run (build container only): the reference env classes vs the CPU oracle
on many randomly drawn configurations (tools/gen_fuzz_fixtures.py's generator), E envs each. Prints
every configuration whose trajectories differ; nothing is written. A mismatch found here becomes a
targeted fixture in tools/gen_fuzz_fixtures.py (the oracle is pinned to the GPU kernels by the
committed fixtures, so a configuration the oracle gets right the kernels are then tested on).

    python tools/fuzz_explore.py [num_configs] [seed]
"""
import json
import os
import sys
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "marl-for-im_amd")]
import gen_fixtures as gf  # noqa: E402
import fuzz_configs as gz  # noqa: E402
from golden_io import decode_config  # noqa: E402
from test_oracle_golden import run_oracle  # noqa: E402

KEYS = ["order", "demand", "acquisition", "ship", "inv", "backlog", "order_u", "profit", "obs", "reward"]


def main():
    num = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    classes = gf.import_reference()
    gf.E = 4
    gf.make_inputs = lambda kind, cfg, opts, seed: gz.fuzz_inputs(kind, cfg, opts, seed, 4)
    rs = np.random.RandomState(seed)
    kinds = ["IM", "MAIM", "IM_div", "MAIM_div"]
    bad = 0
    for idx in range(num):
        kind = kinds[idx % 4]
        cfg = gz.rand_config(rs, kind, int(rs.randint(5)))
        if cfg["inv_max"].max() > 1000:      # keep the oracle's literal split loop fast
            cfg["inv_max"] = np.minimum(cfg["inv_max"], 1000.0)
            cfg["init_inv"] = np.minimum(cfg["init_inv"], cfg["inv_max"])
        cfg = gz.maybe_order_max(rs, kind, cfg)
        opts = {"noisy": 0.3} if rs.rand() < 0.25 else {}
        gf.T = cfg["num_periods"]
        try:
            ref = gf.run_case(classes, "x", kind, cfg, opts, seed=idx)
            meta = json.loads(str(ref.pop("meta")))
            meta["config"] = decode_config(meta["config"])
            if (ref["err"] >= 0).any():
                print("cfg %d %s: reference raised (skipped)" % (idx, kind))
                continue
            obs0, out, _ = run_oracle(meta, ref)
            msgs = []
            if not np.array_equal(obs0, ref["obs0"]):
                msgs.append("obs0")
            for k in KEYS + (["ship_to", "backlog_to"] if kind.endswith("div") else []):
                r = ref[k] if k != "reward" else ref[k][..., :out[k].shape[-1]]
                if not np.array_equal(out[k], r):
                    msgs.append(k)
            if msgs:
                bad += 1
                print("MISMATCH cfg %d %s %s: %s" % (idx, kind, opts, msgs))
                print("   ", {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in cfg.items()})
        except Exception:
            bad += 1
            print("ERROR cfg %d %s" % (idx, kind))
            traceback.print_exc()
    print("done: %d configs, %d mismatches" % (num, bad))


if __name__ == "__main__":
    main()
