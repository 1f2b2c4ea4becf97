# round-5: per-period step durations in the graph-replayed window (kernel trace), table on / off
set -o pipefail
O=${1:-gpurun_out/r5w}; mkdir -p $O
export TMPDIR=/tmp
for d in 1 0; do
  for c in "C4" "C2 --n-envs 131072"; do
    t=$(echo $c | tr -d ' -')_$d
    IMENV_DTAB=$d timeout -k 10 240 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/$t -o p --output-format csv -- python bench.py --config $c --no-cpu-baseline --no-alt-store --no-alt-obs --steps 120 --warmup 30 > $O/$t.json 2> $O/$t.err || exit 1
    echo "== $t $(python -c "import json; d=json.load(open('$O/$t.json')); print(d['roofline']['kernel_us'], d.get('launch'))")"; python tools/trace_by_period.py $O/$t/p_kernel_trace.csv | tail -4
  done
done
