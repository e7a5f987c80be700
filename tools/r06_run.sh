#!/bin/bash
# One GPU session of round 6 (tools/r06_run.sh STEP...): each step is bounded
# by its own timeout; an ordinary failure (rc 1) lets the next step run, a
# time limit, abort, segfault or anything else ends the session there.
# Outputs under gpurun_out/r06/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r06
mkdir -p $O
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
for step in "$@"; do
  case "$step" in
    gputests) timeout -k 10 900 $T -m gpu tests > $O/gputests.log 2>&1 ;;
    smoke)    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    soaknew)  # fresh seeds: ZSCRC_SOAK_BASE=100000
              ZSCRC_SOAK_BASE=100000 ZSCRC_SOAK_SEEDS=250 ZSCRC_SOAK_COMMITS=240 ZSCRC_SOAK_CONSISTENT=60 \
                timeout -k 10 900 $T tests/test_gpu_soak.py tests/test_gpu_consistent.py -k "random" \
                > $O/soaknew.log 2>&1 ;;
    cpass)    timeout -k 10 600 $T tests/test_gpu_consistent.py > $O/cpass_tests.log 2>&1 ;;
    soaklong) ZSCRC_SOAK_SEEDS=250 ZSCRC_SOAK_COMMITS=240 ZSCRC_SOAK_CONSISTENT=60 timeout -k 10 900 \
                $T tests/test_gpu_soak.py tests/test_gpu_consistent.py -k "random" > $O/soaklong.log 2>&1 ;;
    bench2|bench3|bench4|bench5)
              timeout -k 10 900 python bench.py --workload config${step#bench} >> $O/$step.jsonl 2>> $O/$step.err ;;
    bench2q|bench3q|bench4q|bench5q)   # GPU part only
              c=${step#bench}; c=${c%q}
              timeout -k 10 600 python bench.py --workload config$c --no-cpu --no-e2e >> $O/$step.jsonl \
                2>> $O/$step.err ;;
    trace2|trace3|trace4|trace5)
              c=config${step#trace}
              ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d $R/$O/trace_$c -o run -- python3 $R/bench.py --workload $c --no-cpu --no-e2e \
                  > $R/$O/trace_$c.json 2> $R/$O/trace_$c.err ) ;;
    traffic2|traffic3|traffic4|traffic5)   # FETCH_SIZE and WRITE_SIZE passes, 5 passes each
              c=config${step#traffic}
              bash tools/pmc_traffic.sh $c 5 ;;
    rehearse3)
              BENCH_SHARE_GPU=1 BENCH_DIST=gloo timeout -k 10 600 python bench.py --gpus 2 --workload config3 \
                --no-cpu > $O/rehearse3_n2.json 2> $O/rehearse3_n2.err ;;
    rehearse5)
              BENCH_SHARE_GPU=1 BENCH_DIST=gloo timeout -k 10 900 python bench.py --gpus 2 --workload config5 \
                --no-cpu > $O/rehearse5_n2.json 2> $O/rehearse5_n2.err ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc" | tee -a $O/steps.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
