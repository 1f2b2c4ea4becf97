#!/bin/bash
# GPU-box check of the plan replay: its GPU tests, then tools/bench_plan.py lines and a kernel trace.
OUT=${1:-gpurun_out/plan}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py tests/test_base_stock_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_plan.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_plan.log; exit 1; }
tail -2 $OUT/pytest_plan.log
timeout -k 10 200 python tools/bench_plan.py > $OUT/bench_SHLP8_f64.json 2> $OUT/bench_SHLP8_f64.err &&
timeout -k 10 200 python tools/bench_plan.py --no-cpu --f32 > $OUT/bench_SHLP8_f32.json 2>> $OUT/bench.err &&
timeout -k 10 200 python tools/bench_plan.py --no-cpu --config SHLP4 > $OUT/bench_SHLP4_f64.json 2>> $OUT/bench.err &&
timeout -k 10 200 python tools/bench_plan.py --no-cpu --config SHLP_div1 > $OUT/bench_div1_f64.json 2>> $OUT/bench.err &&
timeout -k 10 200 python tools/bench_plan.py --no-cpu --config SHLP4 --layout shared --plans 64 --scenarios 65536 --drawn --no-rewards > $OUT/bench_SHLP4_shared.json 2>> $OUT/bench.err &&
timeout -k 10 200 python tools/bench_rollout.py --no-cpu > $OUT/bench_rollout_IM.json 2>> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o p --output-format csv -- python tools/bench_plan.py --no-cpu > $OUT/bench_prof.json 2> $OUT/bench_prof.err
rc=$?
for f in $OUT/bench_*.json; do echo "$f: $(head -c 400 $f)"; done
echo "gpu_plan rc=$rc"
exit $rc
