#!/bin/bash
# Run one gpurun call, retrying only while the pod has no free GPU slot / box (gpurun exit code 3: nothing ran,
# nothing charged).  Any other outcome, success or failure, is final.
#   scripts/gpurun_retry.sh OUT TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 ${TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -qE "slot\(s\) on this pod are busy|no free box right now" "$OUT"; then break; fi
  sleep ${WAIT:-120}
done
echo "done rc=$rc" >> "$OUT"
