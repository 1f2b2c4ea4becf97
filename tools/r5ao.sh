# round-5: with the load fence, does the hand-over now pay for C4 (two retailers) or C3 (262,144 envs)?
set -o pipefail
O=${1:-gpurun_out/r5ao}; mkdir -p $O
timeout -k 10 900 bash tools/ab_multi.sh $O/ab 3 "--config C4|--config C3|--config C2 --n-envs 262144" \
  "dflt=IMENV_AB=1" "dtab=IMENV_DTAB=1" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
