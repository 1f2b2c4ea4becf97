#!/bin/bash
# Round-3: bench lines with the host-lead spin (bench.py lead_spin) for C4 / C3 at their BASELINE
# sizes (3x each) and the metric's C2 line, with the PMC summaries of this kernel in profiles/pmc_configs.
OUT=${1:-gpurun_out/final_c}
export TMPDIR=/tmp
mkdir -p $OUT
for r in 1 2 3; do
  for c in C4 C3; do
    timeout -k 10 240 python bench.py --config $c --steps 150 --warmup 30 > $OUT/bench_${c}_$r.json 2> $OUT/bench_${c}_$r.err || { echo "bench $c failed"; exit 1; }
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/final_c/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, "%.4g" % d["value"], d["ms_per_step"], r["kernel_us"], r["frac"], r["traffic"], json.dumps(r.get("launch_pacing")))
PY
echo "final_c done"
