# round-5: the load fence + scalar episode-word load (old Philox word select): parity, A/B against no
# fence, then counters for every bench kernel tag (the device-source hash changed)
set -o pipefail
O=${1:-gpurun_out/r5ak}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_drawn_fuzz_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "philox or traffic or drawn or continue" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 1200 bash tools/ab_multi.sh $O/ab 2 "--config C2 --n-envs 131072|--config C4|--config C3|--config C2" \
  "cur=IMENV_AB=1" "nofence=IMENV_JIT_OPTS=-DIMENV_LOAD_FENCE=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
CONFIGS="C2:131072 C2:1048576 C2:1048576:o64 C4:131072 C3:262144" timeout -k 10 1200 bash tools/profile_configs.sh $O/cfgprof > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
for c in C2_131072 C2_1048576 C2_1048576_o64 C4_131072 C3_262144; do python -c "import json; d=json.load(open('$O/cfgprof/$c/summary.json')); print('$c', round(d['hbm_bytes_per_launch']/d['algorithmic_bytes_per_launch'],4), d['trace_avg_ns'])"; done
