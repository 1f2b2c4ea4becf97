#!/bin/bash
# GPU-box iteration loop: parity tests, then bench lines for the configs named in $CONFIGS (default C2).
OUT=${1:-gpurun_out/quick}
CONFIGS=${CONFIGS:-C2}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for c in $CONFIGS; do
  timeout -k 10 300 python bench.py --config $c --n-envs 1048576 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); r=d['roofline']; print('$c', d['value'], r['kernel_us'], r['frac'], r['kernel'])"
done
