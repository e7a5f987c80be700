bash tools/gpu_session.sh \
 "t_runs:300:python -u -m pytest tests/test_gpu_runs.py tests/test_gpu_zsfile.py tests/test_gpu_consistent.py -x -q --timeout 120 --timeout-method thread" \
 "ab_opt:400:AB_CASES=config4_verify,config4_verdict,config4_write,config4_write_nocrc python tools/opt_ab.py 0 2048 32768"
