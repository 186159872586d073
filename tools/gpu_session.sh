#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box, each under its own time limit.
# A step that faults, aborts, segfaults or times out ends the session (no
# further GPU work); an ordinary test failure (exit 1) does not.
# usage: tools/gpu_session.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (${secs}s) $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  case $rc in
    0|1|2|3|5) ;;   # success / test failures / usage: keep going
    *) echo "stopping session after rc=$rc" | tee -a gpurun_out/session.log; exit $rc ;;
  esac
done
