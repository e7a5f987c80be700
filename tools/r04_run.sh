#!/bin/bash
# One GPU session of round 4 (tools/r04_run.sh STEP...): each step is bounded
# by its own timeout and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest --maxfail=10 -q --timeout 300 --timeout-method thread"
for step in "$@"; do
  case "$step" in
    parity)   timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_cpu_written.py tests/test_gpu_runs.py \
                > gpurun_out/parity.log 2>&1 ;;
    newtests) timeout -k 10 600 $T tests/test_gpu_fill.py tests/test_gpu_cpu_written.py tests/test_gpu_repack.py tests/test_gpu_longspans.py \
                tests/test_gpu_consistent.py tests/test_gpu_append.py tests/test_gpu_files.py \
                tests/test_gpu_parity.py > gpurun_out/newtests.log 2>&1 ;;
    gputests) timeout -k 10 900 $T -m gpu tests > gpurun_out/gputests.log 2>&1 ;;
    smoke)    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench2|bench3|bench4|bench5)
              timeout -k 10 600 python bench.py --workload config${step#bench} > gpurun_out/$step.json \
                2> gpurun_out/$step.err ;;
    bench4s)  ZSCRC_OPT=4194304 timeout -k 10 600 python bench.py --workload config4 --no-e2e --no-cpu \
                >> gpurun_out/bench4s.jsonl 2>> gpurun_out/bench4s.err ;;
    bench4q)  timeout -k 10 600 python bench.py --workload config4 --no-e2e --no-cpu \
                >> gpurun_out/bench4q.jsonl 2>> gpurun_out/bench4q.err ;;
    bench5q|bench5s|bench5x)   # config 5: default / static commit rounds (1 << 22) / static span segments (1 << 26)
              case "$step" in bench5q) o=0 ;; bench5s) o=4194304 ;; bench5x) o=67108864 ;; esac
              ZSCRC_OPT=$o timeout -k 10 600 python bench.py --workload config5 --no-cpu \
                >> gpurun_out/$step.jsonl 2>> gpurun_out/$step.err ;;
    abspan)   AB_CASES=span_3GiB,spans_config5 timeout -k 10 600 python tools/opt_ab.py 0 67108864 \
                > gpurun_out/abspan.jsonl 2> gpurun_out/abspan.err ;;
    pmc4box)  timeout -k 10 180 python -c "import json, bench; print(json.dumps(bench.box_info(0)))" > gpurun_out/box4.json \
                2> gpurun_out/box4.err && bash tools/pmc_case.sh config4 ;;
    pmc2box)  timeout -k 10 180 python -c "import json, bench; print(json.dumps(bench.box_info(0)))" > gpurun_out/box.json \
                2> gpurun_out/box.err && bash tools/pmc_case.sh config2 && bash tools/pmc_case.sh config3 ;;
    nbseq)    bash tools/probes/nb_seq.sh ;;
    nbforms)  timeout -k 10 300 python tools/probes/nb_forms.py > gpurun_out/nb_forms.json 2> gpurun_out/nb_forms.err ;;
    nbmix)    ( cd /tmp && export TMPDIR=/tmp && C4NB_MODE=mixed timeout -k 10 300 rocprofv3 --kernel-trace --stats \
                --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/nbmix -o run -- \
                python3 $GRAFT_REPO_ROOT/tools/prof_case.py config4nb 90 > $GRAFT_REPO_ROOT/gpurun_out/nbmix.log 2>&1 ) && \
              python tools/probes/nb_mixed_summary.py gpurun_out/nbmix 15 > gpurun_out/nbmix.json ;;
    cphases)  timeout -k 10 300 python tools/probes/classify_phases.py > gpurun_out/classify_phases.jsonl \
                2> gpurun_out/classify_phases.err ;;
    xdeal)    timeout -k 10 600 python tools/probes/xdeal_ab.py > gpurun_out/xdeal_ab.jsonl 2> gpurun_out/xdeal_ab.err ;;
    xdealnb)  XD_NB=1 timeout -k 10 600 python tools/probes/xdeal_ab.py 0 2 4 8 16 > gpurun_out/xdeal_nb.jsonl \
                2> gpurun_out/xdeal_nb.err ;;
    abnb)     AB_CASES=config4_nb timeout -k 10 600 python tools/opt_ab.py 0 67108864 \
                > gpurun_out/abnb.jsonl 2> gpurun_out/abnb.err ;;
    abonly3)  AB_CASES=config4_nb_verdict,config4_nb timeout -k 10 600 python tools/opt_ab.py 0 268435456 \
                > gpurun_out/abonly3.jsonl 2> gpurun_out/abonly3.err ;;
    longtests) timeout -k 10 600 $T tests/test_gpu_longspans.py > gpurun_out/longtests.log 2>&1 ;;
    tracebench) bash tools/trace_bench.sh config3 config4 config2 config5 ;;
    trace45)  bash tools/trace_bench.sh config4 config5 ;;
    traffic45) bash tools/pmc_traffic.sh config4 5 && bash tools/pmc_traffic.sh config4w 5 && bash tools/pmc_traffic.sh config5 5 ;;
    spantests) timeout -k 10 600 $T tests/test_gpu_stream.py tests/test_gpu_parity.py -k "span" \
                > gpurun_out/spantests.log 2>&1 ;;
    fillsweep) timeout -k 10 600 python tools/probes/fill_sweep.py > gpurun_out/fill_sweep.jsonl 2> gpurun_out/fill_sweep.err ;;
    rehearse3)
              BENCH_SHARE_GPU=1 BENCH_DIST=gloo timeout -k 10 600 python bench.py --gpus 2 --workload config3 \
                --no-cpu > gpurun_out/rehearse3_n2.json 2> gpurun_out/rehearse3_n2.err ;;
    rehearse5)
              BENCH_SHARE_GPU=1 BENCH_DIST=gloo timeout -k 10 900 python bench.py --gpus 2 --workload config5 \
                --no-cpu > gpurun_out/rehearse5_n2.json 2> gpurun_out/rehearse5_n2.err ;;
    rehearse5x8)
              BENCH_SHARE_GPU=1 BENCH_DIST=gloo timeout -k 10 900 python bench.py --gpus 8 --workload config5 \
                --no-cpu --packed-mib 1024 --finalised 256 > gpurun_out/rehearse5_n8.json \
                2> gpurun_out/rehearse5_n8.err ;;
    cwaves)   timeout -k 10 600 python tools/probes/commit_waves.py > gpurun_out/commit_waves.jsonl 2> gpurun_out/commit_waves.err ;;
    ab4split) AB_CASES=config4_verdict,config4_crcs,config4_write,config4_verify timeout -k 10 600 python tools/opt_ab.py \
                0 536870912 > gpurun_out/ab4split.jsonl 2> gpurun_out/ab4split.err ;;
    ab4inl)   AB_CASES=config4_verdict,config4_crcs,config4_write,config4_verify timeout -k 10 600 python tools/opt_ab.py \
                0 16384 536870912 > gpurun_out/ab4inl.jsonl 2> gpurun_out/ab4inl.err ;;
    ab4final) AB_CASES=config4_verdict,config4_crcs,config4_write,config4_verify timeout -k 10 600 python tools/opt_ab.py \
                0 16384 2147483648 536870912 > gpurun_out/ab4final.jsonl 2> gpurun_out/ab4final.err ;;
    ab4tail)  AB_CASES=config4_verdict,config4_crcs,config4_write,config4_verify timeout -k 10 600 python tools/opt_ab.py \
                0 2147483648 2147484160 > gpurun_out/ab4tail.jsonl 2> gpurun_out/ab4tail.err ;;
    bench4t)  ZSCRC_OPT=2147483648 timeout -k 10 600 python bench.py --workload config4 --no-e2e --no-cpu \
                >> gpurun_out/bench4t.jsonl 2> gpurun_out/bench4t.err ;;
    bench4u)  ZSCRC_OPT=2147484160 timeout -k 10 600 python bench.py --workload config4 --no-e2e --no-cpu \
                >> gpurun_out/bench4u.jsonl 2> gpurun_out/bench4u.err ;;
    bench4d)  timeout -k 10 600 python bench.py --workload config4 --no-e2e --no-cpu \
                >> gpurun_out/bench4d.jsonl 2> gpurun_out/bench4d.err ;;
    bench4l)  ZSCRC_OPT=16384 timeout -k 10 600 python bench.py --workload config4 --no-e2e --no-cpu \
                >> gpurun_out/bench4l.jsonl 2> gpurun_out/bench4l.err ;;
    benchdef) timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err ;;
    ab2nt)    AB_CASES=config2_multi32,config2_warm32 timeout -k 10 600 python tools/opt_ab.py 0 64 > gpurun_out/ab2nt.jsonl \
                2> gpurun_out/ab2nt.err ;;
    bench2nt) ZSCRC_OPT=64 timeout -k 10 600 python bench.py --workload config2 --no-cpu >> gpurun_out/bench2nt.jsonl \
                2> gpurun_out/bench2nt.err ;;
    bench2d)  timeout -k 10 600 python bench.py --workload config2 --no-cpu >> gpurun_out/bench2d.jsonl \
                2> gpurun_out/bench2d.err ;;
    sustain45) PC_TIME=1 timeout -k 10 300 python tools/prof_case.py config4 200 > gpurun_out/sustain_config4.json \
                2> gpurun_out/sustain.err && PC_TIME=1 timeout -k 10 300 python tools/prof_case.py config5 200 \
                > gpurun_out/sustain_config5.json 2>> gpurun_out/sustain.err ;;
    bench3d)  timeout -k 10 600 python bench.py --workload config3 --no-cpu >> gpurun_out/bench3d.jsonl 2> gpurun_out/bench3d.err ;;
    bench3f)  ZSCRC_OPT=32 timeout -k 10 600 python bench.py --workload config3 --no-cpu >> gpurun_out/bench3f.jsonl \
                2> gpurun_out/bench3f.err ;;
    bench4h)  ZSCRC_LIB_PATH=$PWD/zeroskip_amd/libzscrc_head.so timeout -k 10 600 python bench.py --workload config4 \
                --no-e2e --no-cpu >> gpurun_out/bench4h.jsonl 2> gpurun_out/bench4h.err ;;
    ab4steal) AB_CASES=config4_verdict,config4_crcs,config4_write,config4_verify timeout -k 10 600 python tools/opt_ab.py \
                0 512 16384 > gpurun_out/ab4steal.jsonl 2> gpurun_out/ab4steal.err ;;
    cwavesb)  timeout -k 10 600 python tools/probes/commit_waves.py base > gpurun_out/commit_waves_base.jsonl 2> gpurun_out/commit_waves.err ;;
    ab4ro)    AB_CASES=config4_verdict,config4_crcs,config4_write,config4_verify timeout -k 10 600 python tools/opt_ab.py \
                0 2147483648 536870912 > gpurun_out/ab4ro.jsonl 2> gpurun_out/ab4ro.err ;;
    ab4)      AB_CASES=config4_verdict,config4_write,config4_crcs timeout -k 10 600 python tools/opt_ab.py 0 4194304 \
                > gpurun_out/ab4.jsonl 2> gpurun_out/ab4.err ;;
    ab3)      AB_CASES=config3,fixed_16KiB,fixed_4KiB timeout -k 10 600 python tools/opt_ab.py 0 16777216 \
                > gpurun_out/ab3.jsonl 2> gpurun_out/ab3.err ;;
    ab3p)     for P in 8 32; do ZSCRC_QDYN_P=$P AB_CASES=config3 timeout -k 10 300 python tools/opt_ab.py 0 16777216 \
                || exit $?; done > gpurun_out/ab3p.jsonl 2> gpurun_out/ab3p.err ;;
    spreadq)  WS_OPT=16777216 timeout -k 10 600 python tools/probes/wave_spread.py > gpurun_out/wave_spread_q.jsonl \
                2> gpurun_out/wave_spread_q.err ;;
    ab2)      AB_CASES=config2_multi32 timeout -k 10 600 python tools/opt_ab.py 0 8388608 2097152 \
                > gpurun_out/ab2.jsonl 2> gpurun_out/ab2.err ;;
    pmc4crcs) C4_CRCS=1 bash tools/pmc_traffic.sh config4w 5 ;;
    spread)   timeout -k 10 600 python tools/probes/wave_spread.py > gpurun_out/wave_spread.jsonl 2> gpurun_out/wave_spread.err ;;
    crossover) timeout -k 10 600 python tools/probes/crossover.py > gpurun_out/crossover.jsonl 2> gpurun_out/crossover.err ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc" | tee -a gpurun_out/steps.log
  # a failed test or bench assertion (rc 1) still lets the next steps run;
  # a time limit, abort, segfault or anything else ends the session here
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
