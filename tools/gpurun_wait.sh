#!/bin/bash
# gpurun with waits while no box / slot is free (exit 3 or a transient status: nothing ran, nothing
# charged); any other outcome, failures included, is returned as is.  usage: gpurun_wait.sh TIMEOUT CMD
T=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@"
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q '"status": "transient"' /root/repo/gpurun_out/.last_call.json 2>/dev/null; then exit $rc; fi
  sleep 100
done
exit $rc
