#!/bin/bash
# A/B a knob given as environment assignments: runs bench.py (no CPU baseline) alternately with
# variant A and variant B, R rounds each, and prints one line per run (value, kernel us, frac).
#   tools/ab_env.sh OUT "A-assignments" "B-assignments" [R] [bench args...]
OUT=$1; A=$2; B=$3; R=${4:-3}; shift 4
mkdir -p $OUT
for r in $(seq 1 $R); do
  for v in A B; do
    if [ $v = A ]; then ASG=$A; else ASG=$B; fi
    env $ASG timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python -c "import json; d=json.load(open('$OUT/${v}_$r.json')); r=d['roofline']; print('$v', '$ASG', d['value'], r['kernel_us'], r['frac'])"
  done
done
