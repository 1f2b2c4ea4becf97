# round-5: C5's shard (C2 at 131,072) state layout x block size: 16-byte records vs rows, 64- vs 128-env
# blocks (128-env blocks give each ring row access a whole 128-byte line: no line shared by two blocks)
set -o pipefail
O=${1:-gpurun_out/r5x}; mkdir -p $O
timeout -k 10 600 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072" \
  "rec64=IMENV_AB=1" "rows64=IMENV_REC=0" "rows128=IMENV_REC=0;IMENV_JIT_BS=128" "rec128=IMENV_JIT_BS=128" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
