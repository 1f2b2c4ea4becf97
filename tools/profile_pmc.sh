#!/bin/bash
# PMC passes for the step kernel + calibration kernels (one counter group per pass,
# --pmc only: no sys/runtime trace). Run on the GPU box from the repo root.
set -e
OUT=${1:-gpurun_out/pmc}
export TMPDIR=/tmp
mkdir -p $OUT
python tools/pmc_calib.py build
BENCH="python bench.py --no-cpu-baseline --no-alt-store --steps 60 --warmup 30"
run() { tag=$1; shift; timeout -k 10 240 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/$OUT/$tag -o p --output-format csv -- $CMD > $OUT/$tag.log 2>&1; }
CMD="python tools/pmc_calib.py"; run cal_fetch FETCH_SIZE; run cal_write WRITE_SIZE
CMD=$BENCH; run fetch FETCH_SIZE; run write WRITE_SIZE
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run sq2 SQ_LEVEL_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_FLAT || echo "sq2 pass failed (counter names?)"
python tools/pmc_summary.py $OUT/summary.json 1048576 $OUT/cal_fetch $OUT/cal_write $OUT/fetch $OUT/write $OUT/sq $OUT/tcc $OUT/sq2 --bench-log $OUT/fetch.log > $OUT/summary.log 2>&1
echo "pmc passes done"
