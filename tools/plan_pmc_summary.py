#!/usr/bin/env python3
"""HBM bytes per launch of the plan-replay kernel from tools/profile_plan.sh's passes: FETCH_SIZE /
WRITE_SIZE of imenv_rollout_jit per dispatch, converted with the calibration kernels' factors
(tools/pmc_summary.py), next to the algorithmic bytes of the profiled bench line.

    python tools/plan_pmc_summary.py DIR > summary.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import CAL_BYTES, load  # noqa: E402


def main():
    d = sys.argv[1]
    s = load([os.path.join(d, t) for t in ("cal_fetch", "cal_write", "fetch", "write")])
    fac = {}
    for k, c in (("read_dwordx4", "FETCH_SIZE"), ("write_dwordx4", "WRITE_SIZE")):
        fac[k] = CAL_BYTES / (s[k][c] * 1024.0)
    c = s["imenv_rollout_jit"]
    rd = c["FETCH_SIZE"] * 1024.0 * fac["read_dwordx4"]
    wr = c["WRITE_SIZE"] * 1024.0 * fac["write_dwordx4"]
    bench = None
    for line in open(os.path.join(d, "fetch.log")):
        if line.startswith("{") and '"roofline"' in line:
            bench = json.loads(line)
    steps = bench["config"]["plans"] * bench["config"]["scenarios"] * bench["config"]["num_periods"]
    alg = bench["roofline"]["bytes_per_env_step"] * steps
    print(json.dumps(dict(kernel_info=bench["kernel"], workload=bench["config"], bytes_per_counter_kb_factor=fac,
                          hbm_read_bytes_per_launch=rd, hbm_write_bytes_per_launch=wr,
                          hbm_bytes_per_launch=rd + wr, algorithmic_bytes_per_launch=alg,
                          measured_over_algorithmic=(rd + wr) / alg), indent=1))


if __name__ == "__main__":
    main()
