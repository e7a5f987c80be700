# bench-protocol kernel traces of configs 2-5 with the final round-3 build, each summarised
# against its own line (tools/trace_summary.py), then a plain config 5 line (tail after the
# .zsdb-check cache)
O=gpurun_out/trace_bench
bash tools/gpu_session.sh \
 "trace:900:bash tools/trace_bench.sh config2 config3 config4 config5" \
 "sum:60:python tools/trace_summary.py $O/config2 zs::multi64_kernel 64 2 > $O/config2_summary.json && python tools/trace_summary.py $O/config3 > $O/config3_summary.json && python tools/trace_summary.py $O/config4 > $O/config4_summary.json && python tools/trace_summary.py $O/config5 > $O/config5_summary.json && cat $O/*_summary.json" \
 "bench5:300:python bench.py --workload config5 --no-cpu" \
 "bench2:300:python bench.py --workload config2 --no-cpu"
