# full GPU suite after the fold merge / classify-zeroed verdict counter; config 4 line; NOTBATCHED sequence
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench4:300:python bench.py --workload config4 --no-cpu --no-e2e" \
 "nbtrace:200:cd /tmp && rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/nbtrace2 -o run -- python3 $R/tools/prof_case.py config4nb 20 > $R/gpurun_out/nbtrace2.log 2>&1 && cd $R && python tools/seq_trace.py gpurun_out/nbtrace2 2"
