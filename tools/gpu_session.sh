#!/bin/bash
# Run GPU steps in order; each under its own time limit.  A step that fails
# with an ordinary test/assert failure (exit 1) does not stop the session; a
# fault, abort, segfault or timeout (any other non-zero code) ends it.
# usage: tools/gpu_session.sh "name:seconds:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
    echo "=== $name ($secs s): $cmd" | tee -a gpurun_out/session.log
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping session after $name (rc=$rc)" | tee -a gpurun_out/session.log
        exit $rc
    fi
done
exit 0
