#!/bin/bash
# Round-3 step-kernel A/B on the box: batched slab write-out (IMENV_SLAB_BATCH, default 1) against the
# per-word loop, interleaved 3x, for BASELINE's configs at their bench sizes; then the parity suites
# that cover the step kernel (golden, drawn, API fuzz, full size) on the new default.
OUT=${1:-gpurun_out/r3g}
export TMPDIR=/tmp
mkdir -p $OUT
show() { python -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['config']['n_envs_per_gpu'], r['kernel_us'], r['frac'])"; }
for r in 1 2 3; do
  for c in C4 C3 C2; do
    for v in 1 0; do
      IMENV_JIT_OPTS="-DIMENV_SLAB_BATCH=$v" timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --no-alt-store --no-graph --steps 90 --warmup 30 > $OUT/${c}_b${v}_$r.json 2> $OUT/${c}_b${v}_$r.err || { echo "bench failed $c $v"; exit 1; }
      show $OUT/${c}_b${v}_$r.json "$c batch=$v"
    done
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fuzz_gpu.py tests/test_api_fuzz_gpu.py tests/test_gpu_fullsize.py tests/test_adaptors_gpu.py tests/test_c_abi_gpu.py tests/test_jit_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
echo "r3g done"
bash tools/gpu_r3h.sh || exit 1
