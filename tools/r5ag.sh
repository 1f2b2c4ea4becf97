# round-5: why the branch-free Philox word select is 2-7x slower on the GPU: parity, then SQ counters of
# the new vs old select at the metric's 2^20
set -o pipefail
O=${1:-gpurun_out/r5ag}; mkdir -p $O
export TMPDIR=/tmp IMENV_DIAG=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "philox and 0" > $O/parity.log 2>&1; echo "parity rc=$?"; tail -3 $O/parity.log
for v in new oldsel; do
  if [ $v = oldsel ]; then export IMENV_JIT_OPTS=-DIMENV_WORD_SWITCH=1; else unset IMENV_JIT_OPTS; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $GRAFT_REPO_ROOT/$O/$v -o p --output-format csv -- python bench.py --config C2 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --steps 30 --warmup 10 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python - $O/$v/p_counter_collection.csv <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "imenv_step" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
done
