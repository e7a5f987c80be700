# Round profile: per config a kernel trace (--stats) and separate FETCH_SIZE /
# WRITE_SIZE passes of tools/prof_case.py (exactly REPS passes each); then
# the bench line of config 3 under rocprofv3 --kernel-trace --stats.
# usage (on the GPU box): bash tools/profile_round.sh [configs...]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof
mkdir -p $O
REPS=${REPS:-10}
for c in ${@:-config2 config3 config4 config5}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${c}_trace -o run -- python3 $R/tools/prof_case.py $c $REPS > $O/${c}_trace.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${c}_fetch -o run -- python3 $R/tools/prof_case.py $c $REPS > $O/${c}_fetch.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${c}_write -o run -- python3 $R/tools/prof_case.py $c $REPS > $O/${c}_write.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_trace -o run -- python3 $R/bench.py > $O/bench.log 2>&1
