#!/bin/bash
# SQ / TA counter passes on the bench workload + the memory-pattern probes (kernel trace).
OUT=${1:-gpurun_out/sq}
export TMPDIR=/tmp
mkdir -p $OUT
BENCH="python bench.py --no-cpu-baseline --steps 60 --warmup 30"
run() { tag=$1; shift; timeout -k 10 240 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/$OUT/$tag -o p --output-format csv -- $BENCH > $OUT/$tag.log 2>&1; }
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA &&
run fetch FETCH_SIZE && run write WRITE_SIZE &&
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/probe -o p --output-format csv -- python tools/probe.py > $OUT/probe.log 2>&1
echo "sq passes rc=$?"
