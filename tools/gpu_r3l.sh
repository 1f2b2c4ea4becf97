#!/bin/bash
# Round-3: buffer loads (IMENV_BUF_LOAD=1) against flat loads over every golden and drawn configuration
# (tools/bench_sweep.py --fuzz), interleaved twice, at 2^20 and at 131,072 envs.
OUT=${1:-gpurun_out/r3l}
export TMPDIR=/tmp
mkdir -p $OUT
for r in 1 2; do
  for n in 1048576 131072; do
    for v in 0 1; do
      IMENV_JIT_OPTS="-DIMENV_BUF_LOAD=$v" timeout -k 10 400 python tools/bench_sweep.py --fuzz --n-envs $n --out $OUT/sw_bl${v}_n${n}_$r.jsonl > $OUT/sw_bl${v}_n${n}_$r.log 2>&1 || { echo "sweep failed $v $n"; tail -5 $OUT/sw_bl${v}_n${n}_$r.log; exit 1; }
      echo "sweep bl=$v n=$n r=$r: $(wc -l < $OUT/sw_bl${v}_n${n}_$r.jsonl) configs"
    done
  done
done
echo "r3l done"
