#!/bin/bash
# One GPU session of round 4 (tools/r04_run.sh STEP...): each step is bounded
# by its own timeout and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for step in "$@"; do
  case "$step" in
    newtests) timeout -k 10 600 $T tests/test_gpu_fill.py tests/test_gpu_cpu_written.py tests/test_gpu_repack.py tests/test_gpu_longspans.py \
                tests/test_gpu_consistent.py > gpurun_out/newtests.log 2>&1 ;;
    gputests) timeout -k 10 900 $T -m gpu tests > gpurun_out/gputests.log 2>&1 ;;
    smoke)    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench2|bench3|bench4|bench5)
              timeout -k 10 600 python bench.py --workload config${step#bench} > gpurun_out/$step.json \
                2> gpurun_out/$step.err ;;
    crossover) timeout -k 10 600 python tools/crossover.py > gpurun_out/crossover.jsonl 2> gpurun_out/crossover.err ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc" | tee -a gpurun_out/steps.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
