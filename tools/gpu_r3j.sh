#!/bin/bash
# Round-3 A/B (interleaved 4x, 150 timed steps each): 64-env blocks and wave-local slab write-out
# against the default, for C4 at 131,072 envs, C3 at 262,144, C2 at 131,072 and at 2^20; then the
# whole GPU suite on the default.
OUT=${1:-gpurun_out/r3j}
export TMPDIR=/tmp
mkdir -p $OUT
show() { python -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['config']['n_envs_per_gpu'], r['kernel_us'], r['frac'], r['kernel'])"; }
B="python bench.py --no-cpu-baseline --no-alt-store --no-graph --steps 150 --warmup 30"
run() {   # tag bs opts bench-args...
  local tag=$1 bs=$2 opts=$3; shift 3
  IMENV_JIT_BS=$bs IMENV_JIT_OPTS="$opts" timeout -k 10 120 $B "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench failed $tag"; return 1; }
  show $OUT/$tag.json "$tag"
}
for r in 1 2 3 4; do
  run C4_def_$r 256 "" --config C4 || exit 1
  run C4_bs64_$r 64 "" --config C4 || exit 1
  run C4_ws_$r 256 "-DIMENV_WAVE_SLAB=1" --config C4 || exit 1
  run C2s_def_$r 256 "" --config C2 --n-envs 131072 || exit 1
  run C2s_bs64_$r 64 "" --config C2 --n-envs 131072 || exit 1
  run C2s_ws_$r 256 "-DIMENV_WAVE_SLAB=1" --config C2 --n-envs 131072 || exit 1
done
for r in 1 2 3; do
  run C3_def_$r 256 "" --config C3 || exit 1
  run C3_ws_$r 256 "-DIMENV_WAVE_SLAB=1" --config C3 || exit 1
  run C2_def_$r 256 "" --config C2 || exit 1
  run C2_ws_$r 256 "-DIMENV_WAVE_SLAB=1" --config C2 || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
echo "r3j done"
