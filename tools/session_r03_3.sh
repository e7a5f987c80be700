bash tools/gpu_session.sh \
 "t_new:300:python -u -m pytest tests/test_gpu_runs.py tests/test_gpu_files.py tests/test_gpu_repack.py -x -q --timeout 120 --timeout-method thread" \
 "runprobe:200:./tools/run_probe" \
 "ab_norun:400:bash tools/lib_ab.sh tools/ab/libzscrc_norun.so config4_verify,config4_write"
