#!/bin/bash
# Round-3 step-kernel A/B on the box: buffer loads off SGPR bases (IMENV_BUF_LOAD=1) against flat
# loads, interleaved 3x, for BASELINE's configs at their bench sizes, plus block sizes for C4; then the
# step-kernel parity suites with the buffer loads on (JIT kernels).
OUT=${1:-gpurun_out/r3h}
export TMPDIR=/tmp
mkdir -p $OUT
show() { python -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['config']['n_envs_per_gpu'], r['kernel_us'], r['frac'])"; }
B="python bench.py --no-cpu-baseline --no-alt-store --no-graph --steps 90 --warmup 30"
for r in 1 2 3; do
  for c in C4 C3 C2; do
    for v in 0 1; do
      IMENV_JIT_OPTS="-DIMENV_BUF_LOAD=$v" timeout -k 10 120 $B --config $c > $OUT/${c}_bl${v}_$r.json 2> $OUT/${c}_bl${v}_$r.err || { echo "bench failed $c $v"; exit 1; }
      show $OUT/${c}_bl${v}_$r.json "$c bufload=$v"
    done
  done
  for bs in 64 128; do
    IMENV_JIT_BS=$bs timeout -k 10 120 $B --config C4 > $OUT/C4_bs${bs}_$r.json 2> $OUT/C4_bs${bs}_$r.err || { echo "bench failed bs $bs"; exit 1; }
    show $OUT/C4_bs${bs}_$r.json "C4 bs=$bs"
  done
done
IMENV_JIT_OPTS="-DIMENV_BUF_LOAD=1" timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fuzz_gpu.py tests/test_api_fuzz_gpu.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_bl1.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu_bl1.log; exit 1; }
tail -n 1 $OUT/pytest_gpu_bl1.log
echo "r3h done"
