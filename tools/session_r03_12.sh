bash tools/gpu_session.sh \
 "t_long:300:python -u -m pytest tests/test_gpu_longspans.py tests/test_gpu_parity.py tests/test_gpu_zsfile.py tests/test_gpu_runs.py tests/test_gpu_files.py tests/test_gpu_consistent.py -x -q --timeout 120 --timeout-method thread" \
 "bench4:300:python bench.py --workload config4 --no-cpu --no-e2e" \
 "trace4:300:bash tools/trace_bench.sh config4"
