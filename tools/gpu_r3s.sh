#!/bin/bash
# Round-3: a larger plan-replay campaign on the final kernels (1,200 new seeds) and the big-capacity
# step campaign (16 cases of tests/fuzz_configs.py's largest scale).
OUT=${1:-gpurun_out/r3s}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 700 python -u tools/fuzz_plan_campaign.py --cases 1200 --start 500000 > $OUT/plan_campaign_1200.log 2>&1 || { echo "plan campaign failed"; tail -20 $OUT/plan_campaign_1200.log; exit 1; }
tail -n 1 $OUT/plan_campaign_1200.log
timeout -k 10 200 python -u tools/fuzz_gpu_campaign.py --cases 16 --start 600000 --big --envs 4 > $OUT/gpu_campaign_big.log 2>&1 || { echo "big campaign failed"; tail -20 $OUT/gpu_campaign_big.log; exit 1; }
tail -n 1 $OUT/gpu_campaign_big.log
echo "r3s done"
