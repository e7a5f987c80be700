# cpass without the two list copies: consistent parity, config 5 line; final-build bench-protocol traces of configs 2, 4, 5
O=gpurun_out/trace_bench
bash tools/gpu_session.sh \
 "t_c:300:python -u -m pytest tests/test_gpu_consistent.py -x -q --timeout 120 --timeout-method thread" \
 "bench5:300:python bench.py --workload config5 --no-cpu" \
 "trace:600:bash tools/trace_bench.sh config2 config4 config5" \
 "sum:60:python tools/trace_summary.py $O/config2 zs::multi64_kernel 64 2 > $O/config2_summary.json && python tools/trace_summary.py $O/config4 > $O/config4_summary.json && python tools/trace_summary.py $O/config5 > $O/config5_summary.json && cat $O/*_summary.json"
