#!/bin/bash
# GPU-box check: parity tests, smoke, default bench line, kernel-trace stats of the bench.
# Each GPU step has its own time limit; steps are chained so the first failure ends the run.
OUT=${1:-gpurun_out/check}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o p --output-format csv -- python bench.py --no-cpu-baseline --no-alt-store > $OUT/bench_prof.json 2> $OUT/bench_prof.err
rc=$?
echo "gpu_check rc=$rc"
exit $rc
