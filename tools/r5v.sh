# round-5: step-kernel durations by period (t % 4) with and without the drawn-demand table (kernel trace)
set -o pipefail
O=${1:-gpurun_out/r5v}; mkdir -p $O
export TMPDIR=/tmp
for d in 1 0; do
  for c in "C4" "C2 --n-envs 131072"; do
    t=$(echo $c | tr -d ' -')_$d
    IMENV_DTAB=$d timeout -k 10 240 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/$t -o p --output-format csv -- python bench.py --config $c --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --steps 120 --warmup 30 > $O/$t.json 2> $O/$t.err || exit 1
    echo "== $t"; python tools/trace_by_period.py $O/$t/p_kernel_trace.csv | tail -4
  done
done
