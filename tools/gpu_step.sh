#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a
# fault-like exit (timeout, abort, segfault, kill). Test failures (exit 1)
# are reported but do not stop later steps.
# usage: tools/gpu_step.sh <seconds> <log> <cmd...>
secs=$1; log=$2; shift 2
mkdir -p "$(dirname "$log")"
echo "=== $(date +%T) step: $* (limit ${secs}s) -> $log"
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "=== rc=$rc"; tail -n 25 "$log"
case $rc in
  0|1|2|5) exit 0 ;;      # pass / test failures / usage / no tests
  *) echo "FATAL step rc=$rc, stopping"; exit 99 ;;
esac
