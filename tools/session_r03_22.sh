cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_session.sh \
 "t_long:400:python -u -m pytest tests/test_gpu_longspans.py tests/test_gpu_zsfile.py tests/test_gpu_runs.py tests/test_gpu_consistent.py -x -q --timeout 120 --timeout-method thread" \
 "nbtrace:200:cd /tmp && rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/nbtrace3 -o run -- python3 $R/tools/prof_case.py config4nb 20 > $R/gpurun_out/nbtrace3.log 2>&1 && cd $R && python tools/seq_trace.py gpurun_out/nbtrace3 2" \
 "bench4:300:python bench.py --workload config4 --no-cpu --no-e2e" \
 "waves:300:WAVES_C3=1 python tools/xparts_waves.py"
