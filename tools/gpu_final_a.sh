#!/bin/bash
# Round-3 final check of the tree on MI355X: whole GPU suite, smoke, the bench line at the driver's
# settings and at the defaults, a kernel trace with stats of the bench, the C3 / C4 lines, and the
# self-launched 2-rank rehearsal on one GPU (plain and --gather).
OUT=${1:-gpurun_out/final}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 180 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o p --output-format csv -- python bench.py --no-cpu-baseline --no-alt-store > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; exit 1; }
for c in C3 C4; do
  timeout -k 10 240 python bench.py --config $c --steps 150 --warmup 30 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_$c -o p --output-format csv -- python bench.py --config $c --no-cpu-baseline --no-alt-store --no-graph --steps 150 --warmup 30 > $OUT/bench_prof_$c.json 2> $OUT/bench_prof_$c.err || { echo "rocprof $c failed"; exit 1; }
done
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 5 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { echo "rehearse failed"; tail -20 $OUT/rehearse2.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --gather --steps 60 --warmup 10 --no-cpu-baseline > $OUT/rehearse2_gather.json 2> $OUT/rehearse2_gather.err || { echo "rehearse gather failed"; tail -20 $OUT/rehearse2_gather.err; exit 1; }
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/final/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unparsed", e); continue
    r = d.get("roofline") or {}
    print(f, d.get("n_gpus"), "%.3e" % d["value"], r.get("kernel_us"), r.get("frac"), r.get("traffic"))
PY
echo "final_a done"
