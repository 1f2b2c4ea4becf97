# round-5: kernel-argument preloading A/B at C5's shard (C2, 131,072 envs) and C4, the GPU suite
set -o pipefail
O=${1:-gpurun_out/r5b}; mkdir -p $O
b() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" > /dev/null 2>&1 || true
}
for i in 1 2 3; do
  for v in "pre_rec" "nopre_rec:IMENV_JIT_PRELOAD=0" "pre_rows:IMENV_REC=0"; do
    name=${v%%:*}; ev=""; [ "$v" != "$name" ] && ev=${v#*:}
    env $ev timeout -k 10 300 python bench.py --n-envs 131072 --steps 150 --warmup 30 --no-cpu-baseline --no-alt-obs --no-alt-store --no-graph > $O/c2s_${name}_$i.json 2> $O/c2s_${name}_$i.err || exit 1
  done
  timeout -k 10 300 python bench.py --config C4 --steps 150 --warmup 30 --no-cpu-baseline --no-alt-obs --no-alt-store --no-graph > $O/c4_$i.json 2> $O/c4_$i.err || exit 1
done
echo benches done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 300 python bench.py --rccl-solo --n-envs 131072 --steps 60 --warmup 10 --no-cpu-baseline > $O/rccl_131072.json 2> $O/rccl_131072.err || exit 1
echo all done
