cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in ${@}; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$c -o run -- python3 $R/tools/prof_case.py $c 10 > $R/gpurun_out/$c.log 2>&1 || exit $?
done
