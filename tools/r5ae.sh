# round-5: GPU suite + smoke after the drawn-fuzz oracle fix, and C5's shard with / without the hand-over
# on the same box (the box-to-box spread of this launch is ~5%)
set -o pipefail
O=${1:-gpurun_out/r5ae}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 180 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --n-envs 131072 --no-cpu-baseline > $O/c5shard_$i.json 2> $O/c5shard_$i.err || exit 1
  IMENV_DTAB=0 timeout -k 10 300 python bench.py --n-envs 131072 --no-cpu-baseline > $O/c5shard_off_$i.json 2> $O/c5shard_off_$i.err || exit 1
done
for f in $O/c5shard*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', d['value'], r['kernel_us'], r['frac'], r['traffic'])"; done
