#!/bin/bash
# One GPU session of round 5 (tools/r05_run.sh STEP...): each step is bounded
# by its own timeout; an ordinary failure (rc 1) lets the next step run, a
# time limit, abort, segfault or anything else ends the session there.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
T="python -u -m pytest --maxfail=10 -q --timeout 300 --timeout-method thread"
for step in "$@"; do
  case "$step" in
    gputests) timeout -k 10 900 $T -m gpu tests > gpurun_out/gputests.log 2>&1 ;;
    soaklong) ZSCRC_SOAK_SEEDS=250 ZSCRC_SOAK_COMMITS=240 ZSCRC_SOAK_CONSISTENT=60 timeout -k 10 900 \
                $T tests/test_gpu_soak.py tests/test_gpu_consistent.py -k "random" > gpurun_out/soaklong.log 2>&1 ;;
    newtests) timeout -k 10 600 $T tests/test_gpu_c_link.py tests/test_gpu_fill.py tests/test_gpu_repack.py \
                tests/test_gpu_mixed.py > gpurun_out/newtests.log 2>&1 ;;
    smoke)    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench2|bench3|bench4|bench5)
              timeout -k 10 900 python bench.py --workload config${step#bench} >> gpurun_out/$step.jsonl \
                2>> gpurun_out/$step.err ;;
    bench3q|bench2q|bench4q|bench5q)   # GPU part only
              c=${step#bench}; c=${c%q}
              timeout -k 10 600 python bench.py --workload config$c --no-cpu --no-e2e >> gpurun_out/$step.jsonl \
                2>> gpurun_out/$step.err ;;
    traffic2|traffic3|traffic4|traffic4w|traffic5)   # FETCH_SIZE and WRITE_SIZE passes, 5 passes each
              c=config${step#traffic}
              bash tools/pmc_traffic.sh $c 5 ;;
    trace2|trace3|trace4|trace5) bash tools/trace_bench.sh config${step#trace} ;;
    bench3f)  ZSCRC_OPT=32 timeout -k 10 600 python bench.py --workload config3 --no-cpu >> gpurun_out/bench3f.jsonl \
                2>> gpurun_out/bench3f.err ;;
    c2bound)  timeout -k 10 300 python tools/probes/config2_bound.py > gpurun_out/config2_bound.jsonl \
                2> gpurun_out/config2_bound.err ;;
    c2tests)  timeout -k 10 600 $T tests/test_gpu_parity.py -k "config2 or multi" > gpurun_out/c2tests.log 2>&1 ;;
    ab4w)     AB_CASES=config4_write_nocrc,config4_write,config4_crcs timeout -k 10 600 python tools/opt_ab.py 0 512 \
                > gpurun_out/ab4w.jsonl 2> gpurun_out/ab4w.err ;;
    cwtests)  timeout -k 10 600 $T tests/test_gpu_cpu_written.py tests/test_gpu_fill.py > gpurun_out/cwtests.log 2>&1 ;;
    bench5sync) BENCH_C5_SYNC=1 timeout -k 10 600 python bench.py --workload config5 --no-cpu >> gpurun_out/bench5sync.jsonl \
                2>> gpurun_out/bench5sync.err ;;
    cstests)  timeout -k 10 600 $T tests/test_gpu_consistent.py > gpurun_out/cstests.log 2>&1 ;;
    rowtail)  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d $R/gpurun_out/rowtail -o run -- python3 $R/tools/probes/c5_row_tail.py 8 > $R/gpurun_out/rowtail.json \
                2> $R/gpurun_out/rowtail.err ) ;;
    rehearse5)
              BENCH_SHARE_GPU=1 BENCH_DIST=gloo timeout -k 10 900 python bench.py --gpus 2 --workload config5 \
                --no-cpu > gpurun_out/rehearse5_n2.json 2> gpurun_out/rehearse5_n2.err ;;
    rehearse3)
              BENCH_SHARE_GPU=1 BENCH_DIST=gloo timeout -k 10 600 python bench.py --gpus 2 --workload config3 \
                --no-cpu > gpurun_out/rehearse3_n2.json 2> gpurun_out/rehearse3_n2.err ;;
    tracenb)  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d $R/gpurun_out/tracenb -o run -- python3 $R/tools/prof_case.py config4nb 20 > $R/gpurun_out/tracenb.log 2>&1 ) ;;
    ab4em)    AB_CASES=config4_verify,config4_crcs,config4_write_nocrc,config4_write,config4_verdict timeout -k 10 600 \
                python tools/opt_ab.py 0 128 > gpurun_out/ab4em.jsonl 2> gpurun_out/ab4em.err ;;
    cputhreads) timeout -k 10 300 python tools/probes/cpu_threads.py > gpurun_out/cpu_threads.jsonl \
                2> gpurun_out/cpu_threads.err ;;
    ab3)      AB_CASES=config3,fixed_16KiB,fixed_4KiB,fixed_1MiB timeout -k 10 600 python tools/opt_ab.py 0 32 \
                > gpurun_out/ab3.jsonl 2> gpurun_out/ab3.err ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc" | tee -a gpurun_out/steps.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
