"""Load the committed golden vectors (tests/golden/*.npz, made by tools/gen_fixtures.py)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def decode_config(cfg):
    out = {}
    for k, v in cfg.items():
        if isinstance(v, dict) and "__nd__" in v:
            out[k] = np.array(v["__nd__"], dtype=v["dtype"])
        elif isinstance(v, dict) and "__conn__" in v:
            out[k] = {int(a): list(b) for a, b in v["__conn__"]}
        else:
            out[k] = v
    return out


NON_CASE = ("base_stock", "cc_obs", "plan_replay")   # gen_base_stock / gen_cc / gen_plan_fixtures.py (own loaders)


def case_names():
    names = (os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))
    return sorted(n for n in names if n not in NON_CASE)


def fuzz_case_names():
    """Randomly drawn configurations (tools/gen_fuzz_fixtures.py), named "fuzz/<case>"."""
    return sorted("fuzz/" + os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "fuzz", "*.npz")))


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    meta = json.loads(str(d.pop("meta")))
    meta["config"] = decode_config(meta["config"])
    return meta, d


def load_kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def adaptor_case_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "adaptor", "*.npz")))


def load_adaptor_case(name):
    z = np.load(os.path.join(GOLDEN, "adaptor", name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    meta = json.loads(str(d.pop("meta")))
    return meta, d


def load_base_stock(fname="base_stock.npz"):
    """tests/golden/base_stock.npz (tools/gen_base_stock_fixtures.py) or plan_replay.npz
    (tools/gen_plan_fixtures.py): {case: {field: array}}, meta."""
    z = np.load(os.path.join(GOLDEN, fname), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    cases = {}
    for k in z.files:
        if k == "meta":
            continue
        c, f = k.split("/")
        cases.setdefault(c, {})[f] = z[k]
    for c in meta:
        meta[c]["config"] = decode_config(meta[c]["config"])
    return meta, cases
