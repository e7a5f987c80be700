bash tools/gpu_session.sh \
 "t_new:300:python -u -m pytest tests/test_gpu_runs.py tests/test_gpu_files.py tests/test_gpu_repack.py -x -q --timeout 120 --timeout-method thread" \
 "runprobe:200:./tools/run_probe" \
 "ab_opt:300:AB_CASES=config4_verify python tools/opt_ab.py 0 2048 4096 8192 12288"
