bash tools/gpu_session.sh \
 "t_cons:300:python -u -m pytest tests/test_gpu_consistent.py tests/test_gpu_parity.py tests/test_gpu_zsfile.py tests/test_gpu_runs.py -x -q --timeout 120 --timeout-method thread" \
 "ab_nb:300:AB_CASES=config4_nb python tools/opt_ab.py 0 65536 131072" \
 "bench5:300:python bench.py --workload config5 --no-cpu" \
 "ab_c2:300:AB_CASES=config2_multi32 python tools/opt_ab.py 0 262144"
