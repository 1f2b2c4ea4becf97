#!/bin/bash
# Round-3 final tree: whole GPU suite and smoke, PMC passes for C4 / C3 / C2 at their bench sizes,
# then the bench lines (C4 / C3 3x each, the metric's line at the driver's settings and the default).
export TMPDIR=/tmp
OUT=gpurun_out/final_d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 180 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
bash tools/gpu_final_b.sh || exit 1
bash tools/gpu_final_c.sh || exit 1
echo "final_d done"
