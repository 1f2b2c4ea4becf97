# round-5: kernel trace of the drawn-demand table's reset (reset kernel + draw kernel durations)
set -o pipefail
O=${1:-gpurun_out/r5s}; mkdir -p $O
export TMPDIR=/tmp
for c in "C2 --n-envs 131072" "C4"; do
  t=$(echo $c | tr -d ' -')
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/$t -o p --output-format csv -- python bench.py --config $c --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --steps 60 --warmup 30 > $O/$t.json 2> $O/$t.err || exit 1
  python - $O/$t/p_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"][:90], r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"])
PY
done
