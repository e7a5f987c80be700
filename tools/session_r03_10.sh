bash tools/gpu_session.sh \
 "runprobe:200:./tools/run_probe" \
 "t_cons:300:python -u -m pytest tests/test_gpu_consistent.py tests/test_gpu_files.py -x -q --timeout 120 --timeout-method thread" \
 "bench5:300:python bench.py --workload config5 --no-cpu" \
 "bench5_one:300:ZSCRC_CPASS_ONE_STREAM=1 python bench.py --workload config5 --no-cpu" \
 "trace4:300:bash tools/trace_bench.sh config4" \
 "repack:400:python tools/repack_bench.py --repack-dir 10000000 > gpurun_out/repack_dir.jsonl"
