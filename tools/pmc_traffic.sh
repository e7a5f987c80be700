# FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 run each) of one tools/prof_case.py config
# usage (GPU box): bash tools/pmc_traffic.sh config4w [REPS]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C=${1:-config4}
N=${2:-5}
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc_${C}_$P -o run -- python3 $R/tools/prof_case.py $C $N > $R/gpurun_out/pmc_${C}_$P.log 2>&1 || exit $?
done
