#!/bin/bash
# Round-end refresh on the GPU box: parity tests, smoke, bench line, kernel-trace stats, PMC HBM bytes,
# every golden config (f32 / f64 observations), BASELINE's C3 / C4, the rollout and the small kernels.
# Each GPU step has its own time limit; the first failure ends the run.
OUT=${1:-gpurun_out/final}
export TMPDIR=/tmp
mkdir -p $OUT
bash tools/profile_pmc.sh $OUT/pmc > $OUT/pmc.log 2>&1 || exit $?
cp $OUT/pmc/summary.json profiles/pmc_step_kernel.json
bash tools/gpu_check.sh $OUT/check || exit $?
timeout -k 10 400 python tools/bench_sweep.py --out $OUT/sweep.jsonl > $OUT/sweep.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_sweep.py --obs-f64 --out $OUT/sweep_f64.jsonl > $OUT/sweep_f64.log 2>&1 || exit $?
bash tools/bench_configs.sh $OUT/configs || exit $?
bash tools/gpu_rollout_check.sh $OUT/rollout || exit $?
timeout -k 10 300 python tools/bench_kernels.py > $OUT/kernels.jsonl 2> $OUT/kernels.err || exit $?
echo "refresh done"
