#!/bin/bash
# Run GPU steps in order; each "name:::seconds:::command" runs under its own timeout.
# A step that crashes (abort/segfault/timeout/kill) ends the sequence; an ordinary failure
# (assertions, non-zero exit) is recorded and the next step runs.
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:::*}"; rest="${spec#*:::}"; secs="${rest%%:::*}"; cmd="${rest#*:::}"
  echo "== $name ($secs s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  case $rc in
    124|134|137|139|143) echo "== stopping after crash/timeout in $name"; exit $rc;;
  esac
done
exit 0
