#!/bin/bash
# Submit one gpurun call, re-submitting it only while the pool has no free box / slot (gpurun exit code 3 or a
# "transient" status: nothing ran, nothing was charged).  Any other outcome -- success or a failure of the command
# itself -- ends the loop; a failing GPU step is never re-run.
#   tools/gpurun_wait.sh LOG TIMEOUT 'command'
log=$1
to=$2
shift 2
for try in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" "$log" && ! grep -q "rc=[0-9]" "$log"; }; then
    echo "[gpurun_wait] try $try: no box ($rc), waiting" >> "$log.tries"
    sleep 150
    continue
  fi
  echo "[gpurun_wait] done rc=$rc after $try tries" >> "$log.tries"
  exit $rc
done
exit 3
