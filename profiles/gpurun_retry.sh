#!/bin/bash
# profiles/gpurun_retry.sh LOG 'command' — submit one gpurun call; resubmit only while the pool answers "no box /
# backing off" (exit 3 or status transient: nothing ran, nothing charged), at most 6 times, 3 minutes apart.  Any
# other outcome (the command ran, passed or failed) ends it.
LOG=${1:?log}; CMD=${2:?command}
for i in 1 2 3 4 5 6; do
    timeout 2500 /usr/local/graft/bin/gpurun --timeout ${GPURUN_LIMIT:-1000} -- "$CMD" > "$LOG" 2>&1
    rc=$?
    if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit $rc; fi
    echo "attempt $i: no box ($rc); waiting" >> "$LOG.attempts"
    sleep 180
done
exit 3
