#!/usr/bin/env bash
# Runs one gpurun call, re-submitting it only while gpurun answers 3 (no box or slot free:
# nothing ran, nothing was charged), every 3 minutes, at most 12 times.  Any other exit code
# (the command ran, failed, or was refused) ends it.  usage: gpurun_wait.sh OUT TIMEOUT 'cmd'
out=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  echo "exit $rc (attempt $i)" >> "$out"
  [ $rc -eq 3 ] || exit $rc
  sleep 180
done
exit 3
