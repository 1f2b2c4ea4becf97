#!/bin/bash
# Round-3 refresh of the next-row kernels that share step_core with the step kernel (the closed-form
# split and integer revenue changed it): base-stock rollout and plan replay bench lines, with a kernel
# trace of the rollout.
OUT=${1:-gpurun_out/r3p}
export TMPDIR=/tmp
mkdir -p $OUT
for c in IM IM8 IM_div1; do
  timeout -k 10 300 python tools/bench_rollout.py --config $c --no-cpu > $OUT/rollout_$c.json 2> $OUT/rollout_$c.err || { echo "rollout $c failed"; exit 1; }
done
for c in SHLP8 SHLP4 SHLP_div1; do
  timeout -k 10 300 python tools/bench_plan.py --config $c --no-cpu > $OUT/plan_$c.json 2> $OUT/plan_$c.err || { echo "plan $c failed"; exit 1; }
done
timeout -k 10 300 python tools/bench_plan.py --config SHLP8 --f32 --no-cpu > $OUT/plan_SHLP8_f32.json 2> $OUT/plan_SHLP8_f32.err || { echo "plan f32 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/trace -o p --output-format csv -- python tools/bench_rollout.py --no-cpu --reps 5 > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_jit_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_jit.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_jit.log; exit 1; }
tail -n 1 $OUT/pytest_jit.log
for f in $OUT/*.json; do echo "$f $(tail -n 1 $f | cut -c1-400)"; done
echo "r3p done"
