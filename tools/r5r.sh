# round-5: drawn-demand table, LDS-staged draw kernel: A/B against the in-kernel draw with the reset cost
set -o pipefail
O=${1:-gpurun_out/r5r}; mkdir -p $O
timeout -k 10 600 bash tools/ab_multi.sh $O/ab 2 "--config C2 --n-envs 131072|--config C4" \
  "dtab=IMENV_AB=1" "nodtab=IMENV_DTAB=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
for f in $O/ab/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['roofline']['reset_us'])"; done
