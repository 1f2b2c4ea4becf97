# round-5: drawn-demand table as a four-period hand-over between steps (no reset-time draw kernel):
# parity (table on / off), A/B on C5's shard and C4, then the whole GPU suite
set -o pipefail
O=${1:-gpurun_out/r5u}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "philox or traffic or sharding or continue" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 600 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072|--config C4" \
  "dtab=IMENV_AB=1" "nodtab=IMENV_DTAB=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
for f in $O/ab/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['roofline']['reset_us'])"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
