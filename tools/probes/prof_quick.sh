# kernel-trace (--stats) of tools/prof_case.py for the given configs (5 passes each)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pq
mkdir -p $O
for c in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o run -- python3 $R/tools/prof_case.py $c 5 > $O/$c.log 2>&1 || exit $?
done
