#!/bin/bash
# Round-3 parity campaigns on the final kernels (the closed-form split, 64-env blocks and the write-out
# changed the step kernel; the rollout shares step_core): 2,000 drawn specifications vs the oracle on
# both step-kernel paths (new seeds), and 400 drawn plan-replay cases.
OUT=${1:-gpurun_out/r3r}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u tools/fuzz_gpu_campaign.py --cases 2000 --start 400000 --mode both > $OUT/gpu_campaign_2000.log 2>&1 || { echo "campaign failed"; tail -20 $OUT/gpu_campaign_2000.log; exit 1; }
tail -n 1 $OUT/gpu_campaign_2000.log
timeout -k 10 400 python -u tools/fuzz_plan_campaign.py --cases 300 --start 400000 > $OUT/plan_campaign_300.log 2>&1 || { echo "plan campaign failed"; tail -20 $OUT/plan_campaign_300.log; exit 1; }
tail -n 1 $OUT/plan_campaign_300.log
echo "r3r done"
