#!/bin/bash
# Tree-path parity suites, then C4 (and C3 / C2) bench lines at BASELINE sizes, R rounds.
OUT=${1:-gpurun_out/tree}; R=${2:-3}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fuzz_gpu.py tests/test_api_fuzz_gpu.py tests/test_gpu_fullsize.py tests/test_base_stock_gpu.py tests/test_plan_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in $(seq 1 $R); do
  for c in C4 C3 C2; do
    timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --no-alt-store --no-graph --steps 90 --warmup 30 > $OUT/bench_${c}_$r.json 2> $OUT/bench_${c}_$r.err || { echo "bench failed $c"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${c}_$r.json')); r=d['roofline']; print('$c', d['value'], r['kernel_us'], r['frac'])"
  done
done
