# round-5: the new Philox word select, eager vs graph launches at 2^20 (r5ai: 28 us eager; r5ah: 18.4 us
# in a graph under the kernel trace)
set -o pipefail
O=${1:-gpurun_out/r5aj}; mkdir -p $O
export TMPDIR=/tmp IMENV_DIAG=1
for v in new oldsel; do
  for l in eager graph; do
    if [ $v = oldsel ]; then export IMENV_JIT_OPTS=-DIMENV_WORD_SWITCH=1; else unset IMENV_JIT_OPTS; fi
    timeout -k 10 180 python bench.py --config C2 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --launch $l > $O/${v}_$l.json 2> $O/${v}_$l.err || { tail -5 $O/${v}_$l.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/${v}_$l.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v $l', r['kernel_us'], r['launch_pacing'].get('gpu_us_per_step_queued'), r['launch_pacing'].get('launch'))"
  done
done
unset IMENV_JIT_OPTS
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/tr_new_eager -o p --output-format csv -- python bench.py --config C2 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --launch eager --steps 60 --warmup 10 > $O/tr_new_eager.json 2> $O/tr_new_eager.err || exit 1
grep -i "imenv_step" $O/tr_new_eager/p_kernel_stats.csv | cut -c1-120
