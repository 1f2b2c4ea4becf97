#!/bin/bash
# HBM bytes of the plan-replay kernel (SHLP_8, float64 per-episode plans, 2^20 scenarios): FETCH_SIZE and
# WRITE_SIZE passes (one counter per pass, --pmc only) over tools/bench_plan.py plus the calibration
# kernels of tools/pmc_calib.py, summarised by tools/plan_pmc_summary.py. Run on the GPU box.
OUT=${1:-gpurun_out/plan_pmc}
export TMPDIR=/tmp
mkdir -p $OUT
python tools/pmc_calib.py build || exit $?
B="python tools/bench_plan.py --no-cpu --reps 3"
run() { tag=$1; shift; timeout -k 10 240 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/$OUT/$tag -o p --output-format csv -- $CMD > $OUT/$tag.log 2>&1; }
CMD="python tools/pmc_calib.py"; run cal_fetch FETCH_SIZE && run cal_write WRITE_SIZE &&
CMD=$B; run fetch FETCH_SIZE && run write WRITE_SIZE &&
python tools/plan_pmc_summary.py $OUT > $OUT/summary.json
rc=$?
cat $OUT/summary.json
exit $rc
