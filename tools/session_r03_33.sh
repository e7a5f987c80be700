# config 2: plain bench line twice, then the same under rocprofv3 kernel tracing (the traced line read 11.9 us/batch)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_session.sh \
 "b2a:300:python bench.py --workload config2 --no-cpu" \
 "b2b:300:python bench.py --workload config2 --no-cpu" \
 "b2t:300:cd /tmp && rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/b2t -o run -- python3 $R/bench.py --workload config2 --no-cpu" \
 "b2c:300:python bench.py --workload config2 --no-cpu"
