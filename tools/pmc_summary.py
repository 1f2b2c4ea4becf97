#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per-kernel mean counter values per dispatch.

    python tools/pmc_summary.py OUT.json N_ENVS DIR [DIR ...] [--bench-log LOG] [--alt-obs-f64]

--alt-obs-f64: summarise the bench line's float64-observation kernel (roofline.alt_obs_f64, the
reference's observation dtype, timed in the same run) instead of its main kernel.

Each DIR is one rocprofv3 -d output (one --pmc pass). Kernel names are shortened
to their template head. If the calibration kernels (tools/pmc_calib.hip, 1 GiB per
dispatch) are present, FETCH_SIZE / WRITE_SIZE -> bytes factors are derived per
access width and the step kernel's HBM traffic per launch is written to OUT.json.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

CAL_BYTES = float(1 << 30)


def short(name):
    m = re.search(r"(imenv_\w+?)(<[^>]*>)?\(", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    if re.match(r"imenv_\w+$", name):       # extern "C" (hipRTC) kernels carry no signature
        return name
    for k in ("read_dwordx4", "read_dword", "write_dwordx4", "write_dword"):
        if re.search(r"\b%s\b" % k, name):
            return k
    return name[:60]


def load(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", ""))
                    acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    acc[k]["_grid"].append(float(row.get("Grid_Size", 0) or 0))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: (sum(v) / len(v)) for c, v in cs.items()}
        out[k]["_dispatch_rows"] = len(cs.get("FETCH_SIZE", cs.get("WRITE_SIZE", [0])))
    return out


def main():
    argv = sys.argv[1:]
    bench = None
    if "--bench-log" in argv:
        i = argv.index("--bench-log")
        bench = argv[i + 1]
        del argv[i:i + 2]
    alt64 = "--alt-obs-f64" in argv
    if alt64:
        argv.remove("--alt-obs-f64")
    trace = None
    if "--trace" in argv:          # rocprofv3 --kernel-trace --stats CSV of the same bench command
        i = argv.index("--trace")
        trace = argv[i + 1]
        del argv[i:i + 2]
    outp = argv[0]
    n_envs = int(argv[1])
    s = load(argv[2:])
    res = {"kernels": s, "n_envs": n_envs}
    if bench:
        # the bench line of the profiled run names the exact kernel variant (bench.py only trusts a
        # PMC summary whose kernel_info equals the kernel it is timing)
        for line in open(bench):
            line = line.strip()
            if line.startswith("{") and '"roofline"' in line:
                rl = json.loads(line)["roofline"]
                if rl["kernel"].startswith("jit-diag:"):
                    # a diagnostic build (IMENV_ABLATE / IMENV_STAMPS: wrong results or extra stores) must never
                    # stand in for the production kernel's traffic
                    raise SystemExit("pmc_summary: refusing a diagnostic kernel build: " + rl["kernel"])
                if alt64:
                    a = rl["alt_obs_f64"]
                    res["kernel_info"] = a["kernel"]
                    res["algorithmic_bytes_per_launch"] = a["bytes_per_env_step"] * n_envs
                else:
                    res["kernel_info"] = rl["kernel"]
                    res["algorithmic_bytes_per_launch"] = rl["bytes_per_launch"]
    fac = {}
    for k, c in (("read_dword", "FETCH_SIZE"), ("read_dwordx4", "FETCH_SIZE"), ("write_dword", "WRITE_SIZE"),
                 ("write_dwordx4", "WRITE_SIZE")):
        if k in s and c in s[k] and s[k][c] > 0:
            fac[k] = CAL_BYTES / (s[k][c] * 1024.0)
    res["bytes_per_counter_kb_factor"] = fac
    step = [k for k in s if k.startswith("imenv_step_kernel") or k.startswith("imenv_step_jit")]
    # the kernel of the summarised line: the float64-observation kernel's name ends in _o64
    step = [k for k in step if k.endswith("_o64") == alt64] or step
    if step and "read_dword" in fac and "write_dword" in fac:
        k = step[0]
        c = s[k]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rd = c["FETCH_SIZE"] * 1024.0 * fac["read_dword"]
            wr = c["WRITE_SIZE"] * 1024.0 * fac["write_dword"]
            res.update(kernel=k, hbm_read_bytes_per_launch=rd, hbm_write_bytes_per_launch=wr,
                       hbm_bytes_per_launch=rd + wr,
                       raw_fetch_kb=c["FETCH_SIZE"], raw_write_kb=c["WRITE_SIZE"])
    if trace and res.get("kernel"):
        import csv
        for row in csv.DictReader(open(trace)):
            if row["Name"].strip('"') == res["kernel"]:
                # the kernel trace's own average duration of the same kernel, for bench.py to print next
                # to its HIP-event time (sub-5 us kernels read high under the trace: profiles/INDEX.md)
                res.update(trace_avg_ns=float(row["AverageNs"]), trace_min_ns=float(row["MinNs"]),
                           trace_calls=int(row["Calls"]))
    with open(outp, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
    for k, c in s.items():
        print(k, {a: round(b, 1) for a, b in c.items()})


if __name__ == "__main__":
    main()
