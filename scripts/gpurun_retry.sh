#!/bin/bash
# gpurun_retry.sh OUT TIMEOUT 'command': run a gpurun call, retrying only while
# gpurun reports no free slot / box (exit 3: nothing ran, nothing charged),
# waiting as long as it asks.  The result (and EXIT code) goes to OUT.
out=$1; to=$2; cmd=$3
for i in $(seq 1 ${TRIES:-12}); do
  timeout $((to + 1800)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > "$out" 2>&1
  rc=$?
  echo "EXIT $rc" >> "$out"
  [ $rc -ne 3 ] && exit $rc
  w=$(grep -o 'retry in [0-9]*s' "$out" | grep -o '[0-9]*' | tail -1)
  sleep $(( ${w:-150} + 30 ))
done
exit 3
