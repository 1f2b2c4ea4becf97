#!/bin/bash
# Round-3: the whole GPU suite with 64-env blocks for small launches (most parity cases are small:
# they now run the 64-env kernels), then C4 at 131,072 envs: default vs ablations (2: no demand draw,
# 8: no profit arithmetic, 16: no decode), interleaved 4x, 150 timed steps.
OUT=${1:-gpurun_out/r3k}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
show() { python -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['config']['n_envs_per_gpu'], r['kernel_us'], r['frac'], r['kernel'])"; }
B="python bench.py --no-cpu-baseline --no-alt-store --no-graph --steps 150 --warmup 30"
for r in 1 2 3 4; do
  for a in 0 2 8 16; do
    IMENV_JIT_OPTS="-DIMENV_ABLATE=$a" timeout -k 10 120 $B --config C4 > $OUT/C4_a${a}_$r.json 2> $OUT/C4_a${a}_$r.err || { echo "bench failed"; exit 1; }
    show $OUT/C4_a${a}_$r.json "C4 ablate=$a"
  done
done
echo "r3k done"
