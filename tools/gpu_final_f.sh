#!/bin/bash
# Round-3 final tree after the split's post-trip fix: the plan-replay campaign that found it (300 cases
# from seed 400000), 500 more step-kernel campaign cases, then the whole GPU suite, smoke, PMC passes
# and bench lines (tools/gpu_final_d.sh).
export TMPDIR=/tmp
OUT=gpurun_out/final_f
mkdir -p $OUT
timeout -k 10 400 python -u tools/fuzz_plan_campaign.py --cases 300 --start 400000 > $OUT/plan_campaign_300.log 2>&1 || { echo "plan campaign failed"; tail -20 $OUT/plan_campaign_300.log; exit 1; }
tail -n 1 $OUT/plan_campaign_300.log
timeout -k 10 300 python -u tools/fuzz_gpu_campaign.py --cases 500 --start 500000 --mode both > $OUT/gpu_campaign_500.log 2>&1 || { echo "campaign failed"; tail -20 $OUT/gpu_campaign_500.log; exit 1; }
tail -n 1 $OUT/gpu_campaign_500.log
rm -rf gpurun_out/final_pmc gpurun_out/final_c gpurun_out/final_d
bash tools/gpu_final_d.sh || exit 1
echo "final_f done"
