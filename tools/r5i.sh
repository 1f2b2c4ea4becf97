# round-5: where the driver-form window's wall time goes at 131,072 envs (bench.py's window diagnostics)
set -o pipefail
O=${1:-gpurun_out/r5i}; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --n-envs 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph > $O/s20_$i.json 2> $O/s20_$i.err || exit 1
done
timeout -k 10 200 python bench.py --n-envs 131072 --steps 150 --warmup 30 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph > $O/s150.json 2> $O/s150.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph > $O/s20_2p20.json 2> $O/s20_2p20.err || exit 1
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel_us'], json.dumps(r['launch_pacing']))"; done
