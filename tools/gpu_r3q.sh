#!/bin/bash
# Round-3 sanity of the final bench.py: the driver's bench line, the C4 line, the bench contract tests.
OUT=${1:-gpurun_out/r3q}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --config C4 --steps 150 --warmup 30 > $OUT/bench_C4.json 2> $OUT/bench_C4.err || { echo "bench C4 failed"; exit 1; }
timeout -k 10 300 python bench.py --config C3 --steps 150 --warmup 30 > $OUT/bench_C3.json 2> $OUT/bench_C3.err || { echo "bench C3 failed"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_bench_contract.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bench.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest_bench.log; exit 1; }
tail -n 1 $OUT/pytest_bench.log
for f in $OUT/*.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', '%.4g' % d['value'], r['kernel_us'], r['frac'], r['traffic'], r['launch_pacing'])"; done
echo "r3q done"
