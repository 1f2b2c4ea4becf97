#!/bin/bash
# Round-3 PMC passes for the three bench configs at their bench sizes (tools/profile_configs.sh):
# FETCH_SIZE / WRITE_SIZE with the gfx950 calibration, SQ and TCC groups, one --pmc pass each.
export TMPDIR=/tmp
CONFIGS="C4:131072 C3:262144 C2:1048576" bash tools/profile_configs.sh gpurun_out/final_pmc || { echo "profile_configs failed"; exit 1; }
for f in gpurun_out/final_pmc/*/summary.json; do
  python -c "import json; d=json.load(open('$f')); print('$f', d['n_envs'], d['kernel_info'], round(d['hbm_bytes_per_launch']), d['algorithmic_bytes_per_launch'], round(d['hbm_bytes_per_launch'] / d['algorithmic_bytes_per_launch'], 4))"
done
echo "final_b done"
