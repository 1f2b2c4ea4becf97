# round-5: interleaved A/B at C5's shard (C2, 131,072 envs) and C4 with kernel-argument preloading on
set -o pipefail
O=${1:-gpurun_out/r5c}; mkdir -p $O
timeout -k 10 1100 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072 --steps 150 --warmup 30|--config C4 --steps 150 --warmup 30" \
  "rows=IMENV_REC=0" "rec=IMENV_REC=1" "rows128=IMENV_REC=0;IMENV_JIT_BS=128" "rec128=IMENV_REC=1;IMENV_JIT_BS=128" \
  "rows_a63=IMENV_REC=0;IMENV_JIT_OPTS=-DIMENV_ABLATE=63" "rec_a63=IMENV_REC=1;IMENV_JIT_OPTS=-DIMENV_ABLATE=63" \
  "rows_nopre=IMENV_REC=0;IMENV_JIT_PRELOAD=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
