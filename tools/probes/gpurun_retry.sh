#!/bin/bash
# Submit one gpurun call; resubmit only when the infrastructure reports a
# transient failure before anything ran (no box / box not prepared / backing
# off).  A call that ran (any exit status of the command) is never repeated.
# usage: tools/probes/gpurun_retry.sh TIMEOUT 'command'
t=$1; shift
for attempt in $(seq 1 40); do
    rm -f gpurun_out/.last_call.json
    /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > /tmp/gpurun_attempt.log 2>&1
    rc=$?
    status=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
    if grep -q "backing off\|stopped responding while being prepared\|no box\|status=transient" /tmp/gpurun_attempt.log && [ "$status" != "ok" ]; then
        wait_s=$(grep -o "retry in [0-9]*s" /tmp/gpurun_attempt.log | grep -o "[0-9]*" | head -1)
        echo "attempt $attempt: transient, retrying in $(( ${wait_s:-60} + 15 ))s"
        { cat /tmp/gpurun_attempt.log; cat gpurun_out/.last_call.json 2>/dev/null; } >> /tmp/gpurun_attempts_all.log
        sleep $(( ${wait_s:-60} + 15 ))
        continue
    fi
    tail -3 /tmp/gpurun_attempt.log
    cat /tmp/gpurun_attempt.log >> /tmp/gpurun_attempts_all.log
    exit $rc
done
echo "gave up after transient failures"
exit 3
