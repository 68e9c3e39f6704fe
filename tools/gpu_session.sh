#!/bin/bash
# One GPU-box session, steps run in order, each under its own time limit; the first step that
# fails ends the session (no retries).  Run through gpurun from the repo root:
#   gpurun --timeout 1100 -- bash tools/gpu_session.sh OUT STEP [STEP ...]
# OUT is a directory under gpurun_out/.  Steps:
#   tests[=PYTEST_K]        the GPU suite (or the tests matching -k PYTEST_K), one process
#   smoke                   __graft_entry__.smoke()
#   bench                   the default bench line (bench.py), summary printed
#   loop=MODEL:B:PREC       the timed loop only (bench.py --loop-only)
#   sweep=MODEL:B:PREC:POL;POL;...   tools/policy_sweep.py, POL = NAME=KEY=VAL[&KEY=VAL] (3 rounds)
#   ab=MODEL:B:PREC:LIB,LIB,...  timed loops of several library builds (tools/build_variant.sh;
#                           "base" = the in-tree library), processes interleaved, 3 rounds
#   pmc=MODEL:B:PREC        PMC traffic + MFMA-busy per op (tools/pmc_traffic.sh)
#   trace=MODEL:B:PREC      rocprofv3 trace of the timed loop regrouped per op (tools/trace_round.sh)
#   roofline                rocprofv3 roofline summaries of every config (tools/round_profile.sh, SKIP_TRACE=1)
#   py=SCRIPT[:ARGS]        python3 SCRIPT ARGS (a tool), ARGS split on commas
set -o pipefail
O=gpurun_out/${1:?out dir}
shift
mkdir -p "$O"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
fail() { echo "step $1 failed"; tail -40 "$2"; exit 1; }
n=0
for step in "$@"; do
  n=$((n + 1))
  key=${step%%=*}
  val=${step#*=}
  [ "$val" = "$step" ] && val=""
  log="$O/${n}_${key}.txt"
  echo "== $step"
  case $key in
    tests)
      if [ -n "$val" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -k "$val" > "$log" 2>&1 || fail "$step" "$log"
      else
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$log" 2>&1 || fail "$step" "$log"
      fi
      tail -2 "$log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || fail "$step" "$log"
      tail -1 "$log" ;;
    bench)
      timeout -k 10 600 python -u bench.py --detail-out "$O/bench_detail.json" > "$O/bench.json" 2> "$log" || fail "$step" "$log"
      tail -c 2000 "$O/bench.json"; echo ;;
    loop)
      IFS=: read -r m b p <<< "$val"
      timeout -k 10 300 python -u bench.py --loop-only --model "$m" --batch "$b" --precision "$p" --steps 20 --warmup 5 > "$log" 2>&1 || fail "$step" "$log"
      tail -1 "$log" ;;
    sweep)
      IFS=: read -r m b p pols <<< "$val"
      args=()
      IFS=';' read -ra pl <<< "$pols"
      for x in "${pl[@]}"; do args+=(--policy "$x"); done
      timeout -k 10 600 python -u tools/policy_sweep.py --model "$m" --batch "$b" --precision "$p" "${args[@]}" > "$log" 2>&1 || fail "$step" "$log"
      cat "$log" ;;
    ab)
      IFS=: read -r m b p libs <<< "$val"
      IFS=',' read -ra ll <<< "$libs"
      for rep in 1 2 3; do
        for lib in "${ll[@]}"; do
          l=""; [ "$lib" != base ] && l=$lib
          SPI_HIP_LIB=$l timeout -k 10 300 python -u bench.py --loop-only --model "$m" --batch "$b" --precision "$p" \
            --steps 20 --warmup 5 > "$log.tmp" 2>&1 || fail "$step" "$log.tmp"
          echo "$(basename "$lib") $rep $(tail -1 "$log.tmp")" | tee -a "$log"
        done
      done ;;
    pmc)
      IFS=: read -r m b p <<< "$val"
      timeout -k 10 900 bash tools/pmc_traffic.sh "$O/pmc_${m}_bs${b}_${p}" --model "$m" --batch "$b" --precision "$p" --iters 12 > "$log" 2>&1 || fail "$step" "$log"
      tail -3 "$log" ;;
    trace)
      timeout -k 10 600 bash tools/trace_round.sh "$val" > "$log" 2>&1 || fail "$step" "$log"
      tail -14 "$log" ;;
    roofline)
      SKIP_TRACE=1 timeout -k 10 1000 bash tools/round_profile.sh > "$log" 2>&1 || fail "$step" "$log"
      tail -3 "$log" ;;
    py)
      script=${val%%:*}
      rest=${val#*:}
      [ "$rest" = "$val" ] && rest=""
      IFS=',' read -ra pa <<< "$rest"
      timeout -k 10 600 python3 -u "$script" "${pa[@]}" > "$log" 2>&1 || fail "$step" "$log"
      tail -30 "$log" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session done"
