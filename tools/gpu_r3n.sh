#!/bin/bash
# Round-3 sweeps with queued launches (tools/bench_sweep.py): the default kernel at 2^20 and 131,072
# envs, float32 and float64 observations; buffer loads vs flat at 131,072 (2x interleaved).
OUT=${1:-gpurun_out/r3n}
export TMPDIR=/tmp
mkdir -p $OUT
sw() { tag=$1; shift; timeout -k 10 400 python tools/bench_sweep.py --fuzz "$@" --out $OUT/$tag.jsonl > $OUT/$tag.log 2>&1 || { echo "sweep $tag failed"; tail -5 $OUT/$tag.log; exit 1; }; echo "$tag: $(wc -l < $OUT/$tag.jsonl) configs"; }
sw f32_n1048576 --n-envs 1048576
sw f64_n1048576 --n-envs 1048576 --obs-f64
for r in 1 2; do
  IMENV_JIT_OPTS="-DIMENV_BUF_LOAD=0" sw bl0_n131072_$r --n-envs 131072
  IMENV_JIT_OPTS="-DIMENV_BUF_LOAD=1" sw bl1_n131072_$r --n-envs 131072
done
echo "r3n done"
