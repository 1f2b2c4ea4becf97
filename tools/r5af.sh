# round-5: the step kernel's loads issued before the demand draw (branch-free Philox word select, scalar
# episode-word load) against the old equality-chain select, which let the compiler place the loads after
# the draw: C5's shard with / without the hand-over, C4, C3 and the metric's 2^20
set -o pipefail
O=${1:-gpurun_out/r5af}; mkdir -p $O
timeout -k 10 1200 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072|--config C4|--config C3|--config C2" \
  "new=IMENV_AB=1" "oldsel=IMENV_JIT_OPTS=-DIMENV_WORD_SWITCH=1" "new_nodtab=IMENV_DTAB=0" "oldsel_nodtab=IMENV_DTAB=0;IMENV_JIT_OPTS=-DIMENV_WORD_SWITCH=1" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
