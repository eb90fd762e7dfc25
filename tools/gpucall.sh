#!/bin/bash
# One parametrised gpurun driver for tests / bench lines / A-B pairs (replaces the per-call scripts of
# rounds 3-4; their numbers live in profiles/).  Usage (on the GPU box, from the repo root):
#   tools/gpucall.sh TAG STEP [STEP ...]
# STEP forms (run in order; the first failure, timeout or crash ends the call):
#   tests:<pytest args>            python -m pytest <args> -x -q  -> gpurun_out/TAG_tN.log
#   bench:[VAR=v,VAR=v:]<args>     python bench.py <args> with the env vars -> gpurun_out/TAG_bN.json
#   prof:<name>:<bench args>       tools/prof.sh <name> <bench args> (eager kernel trace + per-frame summary)
#   pmc:<name>:<bench args>        tools/pmc.sh <name> <bench args> (rocprofv3 --pmc passes)
#   sh:<command>                   any other command, under its own timeout
# Every step runs under `timeout -k 10` (TIMEOUT, default 600 s).
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
T=${TIMEOUT:-600}
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}; rest=${step#*:}
  case $kind in
    tests)
      log=gpurun_out/${TAG}_t$n.log
      timeout -k 10 "$T" python -u -m pytest $rest -x -q --timeout 300 --timeout-method thread > "$log" 2>&1 \
        || { tail -40 "$log"; echo "STEP $n FAILED: $step"; exit 1; }
      tail -1 "$log" ;;
    bench)
      envs=(); args=$rest
      if [[ $rest == *=*:* ]]; then IFS=, read -ra envs <<< "${rest%%:*}"; args=${rest#*:}; fi
      out=gpurun_out/${TAG}_b$n.json
      env "${envs[@]}" timeout -k 10 "$T" python -u bench.py $args > "$out" 2> "${out%.json}.err" \
        || { tail -20 "${out%.json}.err"; echo "STEP $n FAILED: $step"; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('$TAG b$n ${envs[*]}', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), d.get('phases_s_per_step'))" ;;
    prof)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 "$T" bash tools/prof.sh "$name" $args || { echo "STEP $n FAILED: $step"; exit 1; } ;;
    pmc)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 "$T" bash tools/pmc.sh "$name" $args || { echo "STEP $n FAILED: $step"; exit 1; } ;;
    sh)
      timeout -k 10 "$T" bash -c "$rest" || { echo "STEP $n FAILED: $step"; exit 1; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo RC=0
