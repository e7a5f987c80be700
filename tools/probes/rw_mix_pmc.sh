# FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 run each) over rw_mix_probe's
# read, interleaved (mix_g1_sc1) and phased (phase_4) cases, 5 launches each.
# usage (GPU box): bash tools/probes/rw_mix_pmc.sh
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for C in read mix_g1_sc1 phase_4; do
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r06/rwpmc_${C}_$P -o run -- \
      $R/tools/probes/rw_mix_probe $C 5 > $R/gpurun_out/r06/rwpmc_${C}_$P.log 2>&1 || exit $?
  done
done
