#!/usr/bin/env python3
"""profiles/pmc_rollout_kernel.json from a tools/profile_rollout.sh run: the rollout kernel's
SQ counters per launch (PMC passes) and its average duration (kernel-trace stats), tagged with the
kernel variant and workload of the bench line that was profiled.

VALU issue model: the SQ_INSTS_VALU_* class counters split the kernel's vector instructions; each
class is priced with tools/bin/probe_valu's measured cost (SIMD cycles per wave-instruction at the
nominal 2.4 GHz, 8 waves per SIMD) of an instruction that the probe's own PMC pass shows counted in
that class. The probe shows two tiers: ~2.3-2.5 cycles for one- and two-source 32-bit ops (either
encoding) and ~4.2 for float64 / 64-bit ops, three-source ops (v_med3_i32) and v_cndmask with an
SGPR-pair mask. INT32 is priced between v_add_u32 and v_med3_i32; the instructions no class counts
(logic ops, moves, cndmask, float64 max/min/rndne) between v_xor_b32 and the dearest of
v_max_f64 / v_med3_i32 / v_cndmask_b32 / v_mov_b64.
issue_model.frac = modelled issue time / measured kernel time, as a [low, high] pair.

    python tools/rollout_pmc_summary.py OUTDIR > profiles/pmc_rollout_kernel.json
"""
import csv
import glob
import json
import os
import sys


def issue_model(c, probe, kernel_ns):
    cyc = {k: v["simd_cycles_per_wave_instr"] for k, v in probe["ops"].items()}
    f64 = lambda k: c.get("SQ_INSTS_VALU_" + k, 0.0)  # noqa: E731
    fixed = {
        "ADD_F64": (f64("ADD_F64"), cyc["v_add_f64"]),
        "MUL_F64": (f64("MUL_F64"), cyc["v_mul_f64"]),
        "FMA_F64": (f64("FMA_F64"), cyc["v_fma_f64"]),
        "TRANS_F64": (f64("TRANS_F64"), 2 * cyc["v_add_f64"]),      # assumed: not probed, a few per launch
        "CVT": (f64("CVT"), 0.5 * (cyc["v_cvt_f64_i32"] + cyc["v_cvt_i32_f64"])),
        "INT64": (f64("INT64"), cyc["v_mad_u64_u32"]),
    }
    classified = sum(n for n, _ in fixed.values()) + f64("INT32")
    other = c["SQ_INSTS_VALU"] - classified
    base = sum(n * k for n, k in fixed.values())
    lo = base + f64("INT32") * cyc["v_add_u32"] + other * cyc["v_xor_b32"]
    int_hi = max(cyc["v_add_u32_e64"], cyc["v_med3_i32"])
    other_hi = max(cyc[k] for k in ("v_max_f64", "v_med3_i32", "v_cndmask_b32", "v_mov_b64"))
    hi = base + f64("INT32") * int_hi + other * other_hi
    simds = probe["cus"] * 4
    to_ns = lambda cycles: cycles / simds / probe["clock_hz"] * 1e9  # noqa: E731
    return {"classes": {k: n for k, (n, _) in fixed.items()} | {"INT32": f64("INT32"), "unclassified": other},
            "cycles_per_instr": {k: round(v, 3) for k, (_, v) in fixed.items()}
            | {"INT32": [cyc["v_add_u32"], int_hi], "unclassified": [cyc["v_xor_b32"], other_hi]},
            "model_ns": [round(to_ns(lo)), round(to_ns(hi))],
            "frac": [round(to_ns(lo) / kernel_ns, 4), round(to_ns(hi) / kernel_ns, 4)] if kernel_ns else None,
            "source": "tools/probe_valu.hip (probe_valu.json, class mapping from its own PMC pass)"}


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
    probe = os.path.join(d, "probe_valu.json")
    if os.path.exists(probe) and "SQ_INSTS_VALU_INT32" in out["counters"]:
        out["issue_model"] = issue_model(out["counters"], json.load(open(probe)), ns)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
