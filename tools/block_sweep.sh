#!/bin/bash
OUT=gpurun_out/bsw
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "256 1" "128 1" "512 1" "1024 1" "256 2" "128 2" "64 1"; do
  set -- $cfg
  IMENV_JIT_BS=$1 IMENV_JIT_EPT=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 > $OUT/b_$1_$2.json 2>/dev/null || exit $?
  python -c "import json; d=json.load(open('$OUT/b_$1_$2.json')); r=d['roofline']; print('bs=$1 ept=$2', '%.4e'%d['value'], r['kernel_us'], r['kernel'])"
done
