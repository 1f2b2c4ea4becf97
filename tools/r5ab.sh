# round-5: the drawn-demand hand-over beyond 131,072 envs (C2 at 262,144 / 2^20): does it pay where the
# step is HBM-bound?
set -o pipefail
O=${1:-gpurun_out/r5ab}; mkdir -p $O
timeout -k 10 900 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 262144|--config C2" \
  "dflt=IMENV_AB=1" "dtab=IMENV_DTAB=1" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
