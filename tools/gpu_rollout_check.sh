#!/bin/bash
# Rollout-only GPU check: its parity tests, then the bench lines.
OUT=${1:-gpurun_out/rcheck}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_base_stock_gpu.py -x -q > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python tools/bench_rollout.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python tools/bench_rollout.py --config IM_div1 --no-cpu > $OUT/bench_div1.json 2>> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/trace -o p --output-format csv -- python tools/bench_rollout.py --no-cpu --reps 5 > $OUT/trace.log 2>&1
rc=$?
echo "rollout check rc=$rc"
exit $rc
