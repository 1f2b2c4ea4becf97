# round-5 final validation (hand-over + its load fence + scalar episode-word load): GPU suite, smoke,
# bench lines (driver form at 2^20, default, C5 shard x3, C4, C3, RCCL one-rank, 2-rank rehearsal),
# counters for every bench kernel tag, and the fence A/B
set -o pipefail
O=${1:-gpurun_out/r5al}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 180 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --n-envs 131072 --no-cpu-baseline > $O/c5shard_$i.json 2> $O/c5shard_$i.err || exit 1
done
timeout -k 10 300 python bench.py --config C4 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 python bench.py --rccl-solo --n-envs 131072 --steps 60 --warmup 10 --no-cpu-baseline > $O/rccl_131072.json 2> $O/rccl_131072.err || exit 1
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 5 --no-cpu-baseline > $O/rehearse2.json 2> $O/rehearse2.err || exit 1
for f in $O/*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel_us'], r['frac'], r['traffic'], r['launch_pacing'].get('launch'))"; done
CONFIGS="C2:131072 C2:1048576 C2:1048576:o64 C4:131072 C3:262144" timeout -k 10 1200 bash tools/profile_configs.sh $O/cfgprof > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
for c in C2_131072 C2_1048576 C2_1048576_o64 C4_131072 C3_262144; do python -c "import json; d=json.load(open('$O/cfgprof/$c/summary.json')); print('$c', round(d['hbm_bytes_per_launch']/d['algorithmic_bytes_per_launch'],4), d['trace_avg_ns'])"; done
timeout -k 10 900 bash tools/ab_multi.sh $O/ab 2 "--config C2 --n-envs 131072|--config C4|--config C2" \
  "cur=IMENV_AB=1" "nofence=IMENV_JIT_OPTS=-DIMENV_LOAD_FENCE=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
echo all done
