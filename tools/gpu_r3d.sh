#!/bin/bash
# Round-3 batch D: parity of the split / decode changes (tree suites), C4 bench + ablations + stamps.
OUT=gpurun_out/r3d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fuzz_gpu.py tests/test_api_fuzz_gpu.py tests/test_gpu_fullsize.py tests/test_base_stock_gpu.py tests/test_plan_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
  for a in 0 1 2 4 8; do
    IMENV_JIT_OPTS="-DIMENV_ABLATE=$a" timeout -k 10 120 python bench.py --config C4 --no-cpu-baseline --no-alt-store --no-graph --steps 90 --warmup 30 > $OUT/abl_C4_${a}_$r.json 2> $OUT/abl_C4_${a}_$r.err || { echo "ablation failed $a"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/abl_C4_${a}_$r.json')); r=d['roofline']; print('C4 ablate=$a', d['value'], r['kernel_us'], r['frac'])"
  done
done
IMENV_STAMPS=1 IMENV_JIT_OPTS=-DIMENV_STAMPS=1 timeout -k 10 120 python tools/stamp_probe.py --config C4 > $OUT/stamps_C4.json 2> $OUT/stamps_C4.err || { echo "stamps failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/stamps_C4.json')); print(json.dumps(d['launches'][-1]))"
