#!/bin/bash
# The rest of the round-end refresh (after tools/profile_pmc.sh + tools/gpu_check.sh): the rollout
# kernel's PMC / VALU profile, every golden config (f32 / f64 observations), BASELINE's C3 / C4 and the
# small kernels. Each GPU step has its own time limit; the first failure ends the run.
OUT=${1:-gpurun_out/rest}
export TMPDIR=/tmp
mkdir -p $OUT
bash tools/profile_rollout.sh $OUT/rollout > $OUT/rollout.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_sweep.py --out $OUT/sweep.jsonl > $OUT/sweep.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_sweep.py --obs-f64 --out $OUT/sweep_f64.jsonl > $OUT/sweep_f64.log 2>&1 || exit $?
bash tools/bench_configs.sh $OUT/configs || exit $?
timeout -k 10 300 python tools/bench_kernels.py > $OUT/kernels.jsonl 2> $OUT/kernels.err || exit $?
echo "refresh_rest done"
