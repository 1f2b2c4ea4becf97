#!/usr/bin/env python3
"""profiles/pmc_rollout_kernel.json from a tools/profile_rollout.sh run: the rollout kernel's
SQ counters per launch (PMC passes) and its average duration (kernel-trace stats), tagged with the
kernel variant and workload of the bench line that was profiled.

    python tools/rollout_pmc_summary.py OUTDIR > profiles/pmc_rollout_kernel.json
"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    bench = json.loads([l for l in open(os.path.join(d, "bench_prof.json")) if l.startswith("{")][-1])
    acc = {}
    for f in glob.glob(os.path.join(d, "sq*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Kernel_Name"].startswith("imenv_rollout_jit"):
                acc.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    ns = None
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Name"].startswith("imenv_rollout_jit"):
                ns = float(row["AverageNs"])
    out = {"kernel_info": bench["kernel"].split("rollout ")[-1], "policies": bench["config"]["policies"],
           "scenarios": bench["config"]["scenarios"], "num_periods": bench["config"]["num_periods"],
           "kernel_avg_ns": ns, "counters": {k: sum(v) / len(v) for k, v in acc.items()},
           "source": "tools/profile_rollout.sh (separate --pmc passes, --kernel-trace --stats)"}
    out["valu_wave_instr_per_launch"] = out["counters"].get("SQ_INSTS_VALU")
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
