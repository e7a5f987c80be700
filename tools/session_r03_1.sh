bash tools/gpu_session.sh \
 "gputest:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench3:200:python bench.py --no-cpu" \
 "trace:900:bash tools/trace_bench.sh config4 config2 config5" \
 "pmc2:200:bash tools/pmc_case.sh config2" \
 "pmc3:200:bash tools/pmc_case.sh config3" \
 "pmc4:200:bash tools/pmc_case.sh config4"
