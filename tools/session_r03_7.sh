bash tools/gpu_session.sh \
 "t_split:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_zsfile.py tests/test_gpu_runs.py tests/test_gpu_consistent.py -x -q --timeout 120 --timeout-method thread" \
 "ab_nb:300:AB_CASES=config4_nb python tools/opt_ab.py 0 65536 131072" \
 "trace4:300:bash tools/trace_bench.sh config4"
