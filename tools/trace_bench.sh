# rocprofv3 kernel traces of bench.py itself (the driver's protocol: warmup 5,
# 20 timed steps) per workload, so every bench line's kernel_ms can be
# reproduced from profiles/.  usage (GPU box): bash tools/trace_bench.sh config4 ...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace_bench
mkdir -p $O
for c in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/$c -o run -- \
      python3 $R/bench.py --workload $c --no-cpu --no-e2e > $O/$c.json 2> $O/$c.err || exit $?
done
