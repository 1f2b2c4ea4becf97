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


def case_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


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
