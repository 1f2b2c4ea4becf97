#!/bin/bash
# Parity suite, then BASELINE-size bench lines (C4 131,072 / C3 262,144 / C2 2^20; 2 rounds each).
OUT=${1:-gpurun_out/q3}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for r in 1 2; do
  for c in C4 C3 C2; do
    timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --no-alt-store --no-graph --steps 90 --warmup 30 > $OUT/bench_${c}_$r.json 2> $OUT/bench_${c}_$r.err || { echo "bench failed $c"; tail -5 $OUT/bench_${c}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${c}_$r.json')); r=d['roofline']; print('$c', d['value'], r['kernel_us'], r['frac'], r['kernel'][:60])"
  done
done
