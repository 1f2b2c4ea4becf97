# round-5: kernel trace of the new vs old Philox word select at 2^20 (durations in the bench loop)
set -o pipefail
O=${1:-gpurun_out/r5ah}; mkdir -p $O
export TMPDIR=/tmp IMENV_DIAG=1
for v in new oldsel; do
  if [ $v = oldsel ]; then export IMENV_JIT_OPTS=-DIMENV_WORD_SWITCH=1; else unset IMENV_JIT_OPTS; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/$v -o p --output-format csv -- python bench.py --config C2 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --steps 60 --warmup 10 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  grep -i "imenv_step\|reset" $O/$v/p_kernel_stats.csv | cut -c1-160
  python -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', r['kernel_us'], r['launch_pacing'].get('gpu_us_per_step_queued'), r['launch_pacing'].get('launch'))"
done
