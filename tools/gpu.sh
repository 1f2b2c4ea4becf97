#!/bin/bash
# One parameterised script for the GPU box (gpurun): runs the named tasks in order, each GPU step under a
# time limit of its own, and stops at the first failure (nothing more runs on the GPU after it).
#
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash tools/gpu.sh gpurun_out/r4x tests smoke bench
#
# Tasks:
#   tests            the whole GPU suite (pytest -m gpu -x)
#   tests_all        the whole GPU suite without -x (every failure listed; test failures do not stop
#                    the script, a crash or time limit does)
#   smoke            __graft_entry__.smoke()
#   bench            bench.py at the driver's settings (--steps 20 --warmup 5) and at its defaults
#   trace            rocprofv3 --kernel-trace --stats of the default bench command
#   cfg:C:N[:ARGS]   bench line + kernel trace of config C at N envs (ARGS: extra bench flags, commas)
#   pmc:C:N          PMC passes at config C, N envs (tools/profile_configs.sh), summary under OUT/pmc
#   probe_small:N    tools/probe_small.py floors at N envs, plus its kernel trace
#   stamps:C:N       per-wave phase stamps of a diagnostic build (tools/stamp_probe.py)
#   rehearse[:N]     bench.py --gpus N (default 2) --rehearse-one-gpu: every rank on GPU 0 with gloo, the
#                    strong-scaled shards and the gather pass (plain, then --no-gather)
#   pytest:FILES     the GPU tests of the given test files (comma-separated)
#   py:SCRIPT[:ARGS] any python tool, ARGS comma-separated (its stdout to OUT/<script>.log)
#   floors:R         interleaved A/B (tools/ab_multi.sh, R rounds) of the production step kernel and its
#                    access-shape floor (IMENV_ABLATE=63: the same vector loads and stores, no
#                    arithmetic) at C4 / C3 / C2 131,072 / C2 2^20
#   ablate:R         the production kernel beside each ablation alone (decode, split, draw, obs, profit)
#                    and all of them, at C4 and C2 131,072
OUT=${1:?usage: gpu.sh OUTDIR TASK...}
shift
export TMPDIR=/tmp
mkdir -p "$OUT"
R=${GRAFT_REPO_ROOT:-$(pwd)}

fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit 1; }

for task in "$@"; do
  IFS=: read -r kind a b c <<< "$task"
  c=${c//,/ }
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || fail tests "$OUT/pytest_gpu.log"
      tail -n 1 "$OUT/pytest_gpu.log" ;;
    tests_all)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1; rc=$?
      tail -n 3 "$OUT/pytest_gpu.log"
      [ $rc -le 1 ] || fail "tests_all rc=$rc" "$OUT/pytest_gpu.log" ;;
    pytest)
      f=${a//,/ }
      timeout -k 10 600 python -u -m pytest $f -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/pytest_sel.log" 2>&1 || fail "pytest $f" "$OUT/pytest_sel.log"
      tail -n 1 "$OUT/pytest_sel.log" ;;
    smoke)
      timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || fail smoke "$OUT/smoke.log"
      echo "smoke ok" ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" \
        || fail bench "$OUT/bench_driver.err"
      timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || fail bench "$OUT/bench.err"
      echo "bench ok" ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace" -o p --output-format csv -- \
        python bench.py --no-cpu-baseline --no-alt-store --no-alt-obs > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" \
        || fail trace "$OUT/bench_trace.err"
      echo "trace ok" ;;
    cfg)
      D="$OUT/${a}_$b"; mkdir -p "$D"
      timeout -k 10 240 python bench.py --config "$a" --n-envs "$b" --steps 150 --warmup 30 $c > "$D/bench.json" \
        2> "$D/bench.err" || fail "cfg $a $b" "$D/bench.err"
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/$D/trace" -o p --output-format csv -- \
        python bench.py --config "$a" --n-envs "$b" --steps 150 --warmup 30 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph $c \
        > "$D/bench_trace.json" 2> "$D/bench_trace.err" || fail "cfg trace $a $b" "$D/bench_trace.err"
      echo "cfg $a $b ok" ;;
    pmc)
      CONFIGS="$a:$b" timeout -k 10 900 bash tools/profile_configs.sh "$OUT/pmc" > "$OUT/pmc_${a}_${b}.log" 2>&1 \
        || fail "pmc $a $b" "$OUT/pmc_${a}_${b}.log"
      echo "pmc $a $b ok" ;;
    probe_small)
      timeout -k 10 200 python tools/probe_small.py --n-envs "$a" > "$OUT/probe_small_$a.json" 2> "$OUT/probe_small_$a.err" \
        || fail probe_small "$OUT/probe_small_$a.err"
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$OUT/probe_small_$a" -o p --output-format csv -- \
        python tools/probe_small.py --n-envs "$a" > "$OUT/probe_small_trace_$a.json" 2> "$OUT/probe_small_trace_$a.err" \
        || fail "probe_small trace" "$OUT/probe_small_trace_$a.err"
      echo "probe_small $a ok" ;;
    stamps)
      IMENV_DIAG=1 IMENV_STAMPS=1 IMENV_JIT_OPTS=-DIMENV_STAMPS=1 timeout -k 10 200 python tools/stamp_probe.py --config "$a" \
        --n-envs "$b" > "$OUT/stamps_${a}_$b.json" 2> "$OUT/stamps_${a}_$b.err" || fail stamps "$OUT/stamps_${a}_$b.err"
      echo "stamps $a $b ok" ;;
    rehearse)
      w=${a:-2}
      timeout -k 10 300 python bench.py --gpus "$w" --rehearse-one-gpu --steps 20 --warmup 5 > "$OUT/rehearse$w.json" \
        2> "$OUT/rehearse$w.err" || fail rehearse "$OUT/rehearse$w.err"
      timeout -k 10 300 python bench.py --gpus "$w" --rehearse-one-gpu --no-gather --steps 60 --warmup 10 --no-cpu-baseline \
        > "$OUT/rehearse${w}_nogather.json" 2> "$OUT/rehearse${w}_nogather.err" || fail "rehearse no-gather" "$OUT/rehearse${w}_nogather.err"
      echo "rehearse $w ok" ;;
    floors)
      timeout -k 10 1500 bash tools/ab_multi.sh "$OUT/floors" "$a" \
        "--config C4|--config C3|--config C2 --n-envs 131072|--config C2 --steps 60 --warmup 30" \
        "base=IMENV_AB=0" "floor=IMENV_JIT_OPTS=-DIMENV_ABLATE=63" > "$OUT/floors.log" 2>&1 \
        || fail floors "$OUT/floors.log"
      echo "floors ok" ;;
    ablate)
      timeout -k 10 1500 bash tools/ab_multi.sh "$OUT/ablate" "$a" "--config C4|--config C2 --n-envs 131072" \
        "base=IMENV_AB=0" "a63=IMENV_JIT_OPTS=-DIMENV_ABLATE=63" "a16=IMENV_JIT_OPTS=-DIMENV_ABLATE=16" \
        "a1=IMENV_JIT_OPTS=-DIMENV_ABLATE=1" "a2=IMENV_JIT_OPTS=-DIMENV_ABLATE=2" "a4=IMENV_JIT_OPTS=-DIMENV_ABLATE=4" \
        "a8=IMENV_JIT_OPTS=-DIMENV_ABLATE=8" > "$OUT/ablate.log" 2>&1 || fail ablate "$OUT/ablate.log"
      echo "ablate ok" ;;
    py)
      s=$(basename "$a" .py)
      b=${b//,/ }
      timeout -k 10 600 python -u "$a" $b > "$OUT/$s.log" 2>&1 || fail "py $a" "$OUT/$s.log"
      tail -n 2 "$OUT/$s.log" ;;
    *)
      echo "unknown task $task"; exit 2 ;;
  esac
done
echo "gpu.sh done: $*"
