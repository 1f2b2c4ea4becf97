# round-5: counters for C5's shard kernel with the drawn-demand hand-over (new kernel tag), and the
# bench-contract / traffic GPU tests
set -o pipefail
O=${1:-gpurun_out/r5y}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bench_contract.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bench or traffic" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
CONFIGS="C2:131072" timeout -k 10 900 bash tools/profile_configs.sh $O/cfgprof > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -3 $O/prof.log
cat $O/cfgprof/C2_131072/summary.log | tail -30
