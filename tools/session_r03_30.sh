# final build: full GPU suite, smoke, every bench line, the config 3 bench-protocol trace
O=gpurun_out/trace_bench
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench3:300:python bench.py" \
 "trace3:300:bash tools/trace_bench.sh config3 && python tools/trace_summary.py $O/config3 > $O/config3_summary.json && cat $O/config3_summary.json" \
 "bench4:300:python bench.py --workload config4 --no-cpu" \
 "bench5:300:python bench.py --workload config5 --no-cpu" \
 "bench2:300:python bench.py --workload config2 --no-cpu"
