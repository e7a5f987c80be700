bash tools/gpu_session.sh \
 "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench4:300:python bench.py --workload config4" \
 "ab_nb:300:AB_CASES=config4_nb python tools/opt_ab.py 0 65536" \
 "trace4:300:bash tools/trace_bench.sh config4"
