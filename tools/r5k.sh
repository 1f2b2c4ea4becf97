# round-5: graph-submitted timed window (bench.py --launch auto/graph/eager) at 131,072 envs and 2^20
set -o pipefail
O=${1:-gpurun_out/r5k}; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --n-envs 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph > $O/s20_auto_$i.json 2> $O/s20_auto_$i.err || { tail -20 $O/s20_auto_$i.err; exit 1; }
  timeout -k 10 200 python bench.py --n-envs 131072 --steps 150 --warmup 30 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph > $O/s150_auto_$i.json 2> $O/s150_auto_$i.err || exit 1
done
timeout -k 10 200 python bench.py --n-envs 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --launch eager > $O/s20_eager.json 2> $O/s20_eager.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph > $O/s20_2p20_auto.json 2> $O/s20_2p20_auto.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --launch graph > $O/s20_2p20_graph.json 2> $O/s20_2p20_graph.err || exit 1
timeout -k 10 200 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph > $O/c4_s20_auto.json 2> $O/c4_s20_auto.err || exit 1
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel_us'], r['frac'], d['resets_timed'], json.dumps(r['launch_pacing']))"; done
