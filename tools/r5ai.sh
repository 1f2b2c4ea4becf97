# round-5: repeat of r5af's select A/B (whose "new" variants ran 2-7x slow on that box only)
set -o pipefail
O=${1:-gpurun_out/r5ai}; mkdir -p $O
rocm-smi --showuse --showclocks > $O/smi_before.txt 2>&1 || true
timeout -k 10 1200 bash tools/ab_multi.sh $O/ab 2 "--config C2 --n-envs 131072|--config C4|--config C3|--config C2" \
  "new=IMENV_AB=1" "oldsel=IMENV_JIT_OPTS=-DIMENV_WORD_SWITCH=1" "new_nodtab=IMENV_DTAB=0" "oldsel_nodtab=IMENV_DTAB=0;IMENV_JIT_OPTS=-DIMENV_WORD_SWITCH=1" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
