bash tools/gpu_session.sh \
 "t_runs:240:python -u -m pytest tests/test_gpu_runs.py tests/test_gpu_files.py -x -v --timeout 120 --timeout-method thread" \
 "gputest:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "ab_opt:240:AB_CASES=config4_verify,config4_write python tools/opt_ab.py 0 2048" \
 "ab_lib:400:bash tools/lib_ab.sh tools/ab/libzscrc_r02.so config4_verify,config4_write" \
 "pmc4:200:bash tools/pmc_case.sh config4" \
 "pmc4w:200:bash tools/pmc_case.sh config4w" \
 "tr4w:200:bash tools/pmc_traffic.sh config4w" \
 "coop:120:./tools/coop_probe"
