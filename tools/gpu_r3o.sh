#!/bin/bash
# Round-3: FMA order decode with a saturated integer clamp (IMENV_DECODE_FMA=1, default) vs the float64
# clamp, interleaved 4x for C4 / C2 at their bench sizes; then the whole GPU suite on the default.
OUT=${1:-gpurun_out/r3o}
export TMPDIR=/tmp
mkdir -p $OUT
show() { python -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['config']['n_envs_per_gpu'], r['kernel_us'], r['frac'])"; }
B="python bench.py --no-cpu-baseline --no-alt-store --no-graph --steps 150 --warmup 30"
for r in 1 2 3 4; do
  for v in 1 0; do
    IMENV_JIT_OPTS="-DIMENV_DECODE_FMA=$v" timeout -k 10 120 $B --config C4 > $OUT/C4_d${v}_$r.json 2> $OUT/C4_d${v}_$r.err || { echo "bench failed"; exit 1; }
    show $OUT/C4_d${v}_$r.json "C4 decode_fma=$v"
  done
done
for r in 1 2; do
  for v in 1 0; do
    IMENV_JIT_OPTS="-DIMENV_DECODE_FMA=$v" timeout -k 10 120 $B --config C2 > $OUT/C2_d${v}_$r.json 2> $OUT/C2_d${v}_$r.err || { echo "bench failed"; exit 1; }
    show $OUT/C2_d${v}_$r.json "C2 decode_fma=$v"
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
echo "r3o done"
