#!/bin/bash
# One parameterized GPU session (replaces the per-experiment gpu_*.sh files).
#   scripts/gpu_run.sh OUT STEP [STEP ...]
# OUT is a directory under gpurun_out/. Each STEP is NAME=COMMAND: the command
# runs under its own `timeout -k 10` (seconds from MILP_STEP_TIMEOUT, default
# 600, or NAME@SECONDS=COMMAND), with stdout in OUT/NAME.out and stderr in
# OUT/NAME.err. The first failing step ends the session (no GPU work after a
# fault, a crash or a time limit). A heartbeat line every 60 s keeps a long
# step visibly alive.
set -u
out=$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
(while true; do sleep 60; echo "[gpu_run] alive $(date +%T)"; done) &
beat=$!
trap 'kill $beat 2>/dev/null' EXIT
for step in "$@"; do
  name=${step%%=*}
  cmd=${step#*=}
  secs=${MILP_STEP_TIMEOUT:-600}
  if [[ $name == *@* ]]; then
    secs=${name#*@}
    name=${name%%@*}
  fi
  echo "[gpu_run] $(date +%T) step $name (limit ${secs}s): $cmd"
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.out" 2> "$out/$name.err"
  rc=$?
  echo "[gpu_run] $(date +%T) step $name rc=$rc in $(( $(date +%s) - t0 ))s"
  echo "$name rc=$rc s=$(( $(date +%s) - t0 ))" >> "$out/steps.txt"
  tail -n 3 "$out/$name.out" "$out/$name.err"
  if [ $rc -ne 0 ]; then
    echo "[gpu_run] stopping after $name (rc=$rc)"
    exit $rc
  fi
done
