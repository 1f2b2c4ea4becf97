#!/bin/bash
# Rollout kernel: bench lines, kernel-trace stats and SQ counter passes (one counter group per pass,
# --pmc only) plus the VALU issue-cost probe, summarised into $OUT/pmc_rollout_kernel.json. Run on
# the GPU box from the repo root.
OUT=${1:-gpurun_out/rollout}
export TMPDIR=/tmp
mkdir -p $OUT
B="python tools/bench_rollout.py --no-cpu --reps 5"
# instruction-class counters (8 SQ counters: the per-pass limit); tools/bin/probe_valu prices each class
CLASSES="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
mkdir -p tools/bin; test -x tools/bin/probe_valu || hipcc --offload-arch=gfx950 -O3 -o tools/bin/probe_valu tools/probe_valu.hip
timeout -k 10 300 python tools/bench_rollout.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python tools/bench_rollout.py --config IM8 --no-cpu > $OUT/bench_im8.json 2>> $OUT/bench.err &&
timeout -k 10 300 python tools/bench_rollout.py --config IM_div1 --no-cpu > $OUT/bench_div1.json 2>> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/trace -o p --output-format csv -- $B > $OUT/bench_prof.json 2> $OUT/trace.log &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/$OUT/sq1 -o p --output-format csv -- $B > $OUT/sq1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d $GRAFT_REPO_ROOT/$OUT/sq2 -o p --output-format csv -- $B > $OUT/sq2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc $CLASSES -d $GRAFT_REPO_ROOT/$OUT/sq3 -o p --output-format csv -- $B > $OUT/sq3.log 2>&1 &&
timeout -k 10 120 tools/bin/probe_valu > $OUT/probe_valu.json &&
timeout -k 10 120 rocprofv3 --pmc $CLASSES -d $GRAFT_REPO_ROOT/$OUT/probe_pmc -o p --output-format csv -- tools/bin/probe_valu > $OUT/probe_pmc.log 2>&1 &&
python tools/rollout_pmc_summary.py $OUT > $OUT/pmc_rollout_kernel.json
rc=$?
echo "profile_rollout rc=$rc"
exit $rc
