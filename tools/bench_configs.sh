#!/bin/bash
# bench.py over BASELINE's single-GPU configs (C2 default, C3, C4 at their sizes and at 2^20 envs) and a
# kernel-trace of each. Each GPU step has its own limit; the first failure ends the run.
OUT=${1:-gpurun_out/configs}
export TMPDIR=/tmp
mkdir -p $OUT
for c in C3 C4; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 1.0 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  timeout -k 10 300 python bench.py --config $c --n-envs 1048576 --no-cpu-baseline > $OUT/bench_${c}_1M.json 2> $OUT/bench_${c}_1M.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_$c -o p --output-format csv -- python bench.py --config $c --n-envs 1048576 --no-cpu-baseline --no-alt-store --steps 120 > $OUT/bench_prof_$c.json 2> $OUT/bench_prof_$c.err || exit $?
done
echo "bench_configs done"
