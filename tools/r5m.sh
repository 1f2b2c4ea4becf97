# round-5: why the host's per-step enqueue doubles while the GPU runs (eager window at 131,072 envs):
# HIP runtime kernel-argument placement knobs
set -o pipefail
O=${1:-gpurun_out/r5m}; mkdir -p $O
B="python bench.py --n-envs 131072 --steps 150 --warmup 30 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --launch eager"
for v in "default:IMENV_AB=1" "devka0:HIP_FORCE_DEV_KERNARG=0" "devka1:HIP_FORCE_DEV_KERNARG=1" "hdp0:DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0" "fgs1:ROC_USE_FGS_KERNARG=1" "fgs0:ROC_USE_FGS_KERNARG=0" "skipcopy:ROC_SKIP_KERNEL_ARG_COPY=1"; do
  name=${v%%:*}; ev=${v#*:}
  env $ev timeout -k 10 200 $B > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/$name.json')); r=d['roofline']; p=r['launch_pacing']; w=p['window']
print('$name', d['value'], d['ms_per_step'], r['kernel_us'], 'host_cal', p['host_us_per_step'], 'gpu_q', p['gpu_us_per_step_queued'], 'enq/step', round(w['host_enqueue_us']/150,2), 'span', w['gpu_span_us'])"
done
