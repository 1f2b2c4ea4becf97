#!/bin/bash
# Interleaved A/B/C... of knobs, each one environment assignment (its value may hold spaces), per bench config:
#   tools/ab_multi.sh OUT ROUNDS "CFG_ARGS1|CFG_ARGS2" "NAME=VAR=value[;VAR2=value2]" ...
# Each (config, variant) pair runs bench.py (no CPU baseline, no alt-store, no graph) ROUNDS times,
# variants interleaved; one line per run: config, variant, value, kernel us, frac.
OUT=$1; R=$2; CFGS=$3; shift 3
mkdir -p $OUT
# a variant may build a diagnostic kernel (-DIMENV_ABLATE=..., e.g. the access-shape floor with no
# arithmetic): allowed here, and bench.py marks such lines "diagnostic_build"
export IMENV_DIAG=1
IFS='|' read -ra CL <<< "$CFGS"
for ci in "${!CL[@]}"; do
  for r in $(seq 1 $R); do
    for v in "$@"; do
      name=${v%%=*}; asg=${v#*=}
      IFS=';' read -ra AS <<< "$asg"
      f=$OUT/c${ci}_${name}_$r
      env "${AS[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph ${CL[$ci]} > $f.json 2> $f.err || { echo "FAIL $f"; tail -5 $f.err; exit 1; }
      python -c "import json; d=json.load(open('$f.json')); r=d['roofline']; print('${CL[$ci]}', '$name', d['value'], r['kernel_us'], r['frac'])"
    done
  done
done
