# round-5 end check on the committed tree: smoke, the driver-form line and C5's shard / C4 lines with their
# PMC traffic (the committed summaries match the kernel tags)
set -o pipefail
O=${1:-gpurun_out/r5aq}; mkdir -p $O
timeout -k 10 180 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 300 python bench.py --n-envs 131072 --no-cpu-baseline > $O/c5shard.json 2> $O/c5shard.err || exit 1
timeout -k 10 300 python bench.py --config C4 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 1
for f in $O/*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', d['value'], r['kernel_us'], r['frac'], r['traffic'], d['resets_timed'], (r.get('alt_obs_f64') or {}).get('traffic'))"; done
