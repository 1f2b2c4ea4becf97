# round-5: counters for every bench kernel tag after the device-source change (the tag carries its hash)
set -o pipefail
O=${1:-gpurun_out/r5z}; mkdir -p $O
CONFIGS="C2:1048576 C2:1048576:o64 C4:131072 C3:262144" timeout -k 10 1000 bash tools/profile_configs.sh $O/cfgprof > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -5 $O/prof.log
for d in $O/cfgprof/*/; do python -c "import json; d=json.load(open('$d/summary.json')); print('$d', d['kernel_info'][:60], round(d['hbm_bytes_per_launch']/d['algorithmic_bytes_per_launch'],4), d['trace_avg_ns'])"; done
