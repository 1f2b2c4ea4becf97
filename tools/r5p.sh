# round-5: with the launch-bound windows replayed as one graph (clean per-launch times), how much of C5's
# shard and C4 is the in-kernel demand draw (IMENV_ABLATE=2) and all arithmetic (63)?
set -o pipefail
O=${1:-gpurun_out/r5p}; mkdir -p $O
timeout -k 10 900 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072|--config C4" \
  "base=IMENV_AB=1" "nodraw=IMENV_JIT_OPTS=-DIMENV_ABLATE=2" "noarith=IMENV_JIT_OPTS=-DIMENV_ABLATE=63" \
  > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
