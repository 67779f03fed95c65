#!/bin/bash
# Runs one gpurun call, waiting out infrastructure-side unavailability only ("no free box", "backing off",
# box taken away before the command ran: gpurun's transient status, nothing charged). A command that ran
# and failed is never repeated. usage: tools/gpurun_wait.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient"; then
    w=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*"); sleep $(( ${w:-100} + 10 )); continue
  fi
  exit $rc
done
exit 3
