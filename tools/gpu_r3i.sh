#!/bin/bash
# Round-3 step-kernel A/B at BASELINE's small sizes, interleaved 4x: default (256-env blocks, flat
# loads), 64-env blocks, wave-local slab write-out, buffer loads, buffer loads + 64-env blocks; C2 at
# 2^20 for the same variants (3x). Each run: 150 timed steps after 30 warm-up steps.
OUT=${1:-gpurun_out/r3i}
export TMPDIR=/tmp
mkdir -p $OUT
show() { python -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['config']['n_envs_per_gpu'], r['kernel_us'], r['frac'], r['kernel'])"; }
B="python bench.py --no-cpu-baseline --no-alt-store --no-graph --steps 150 --warmup 30"
run() {   # tag config bs opts
  IMENV_JIT_BS=$3 IMENV_JIT_OPTS="$4" timeout -k 10 120 $B --config $2 > $OUT/$1.json 2> $OUT/$1.err || { echo "bench failed $1"; exit 1; }
  show $OUT/$1.json "$1"
}
for r in 1 2 3 4; do
  for c in C4 C3; do
    run ${c}_def_$r $c 256 "" || exit 1
    run ${c}_bs64_$r $c 64 "" || exit 1
    run ${c}_ws_$r $c 256 "-DIMENV_WAVE_SLAB=1" || exit 1
    run ${c}_bl_$r $c 256 "-DIMENV_BUF_LOAD=1" || exit 1
    run ${c}_blbs64_$r $c 64 "-DIMENV_BUF_LOAD=1" || exit 1
  done
done
for r in 1 2 3; do
  run C2_def_$r C2 256 "" || exit 1
  run C2_bs64_$r C2 64 "" || exit 1
  run C2_bl_$r C2 256 "-DIMENV_BUF_LOAD=1" || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
echo "r3i done"
