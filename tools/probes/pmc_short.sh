# SQ counters for the one-lane-per-record kernels (one rocprofv3 pass per set)
# usage: DEPTHS="3 9" STRIDE=320 LEN=312 SHIFT=40 bash tools/probes/pmc_short.sh
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
P3="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  for dp in ${DEPTHS:-3 9}; do
    ZS_DEPTH=$dp ZS_SHIFT=${SHIFT:-40} timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc_d${dp}_$i -o run -- python3 $R/tools/probes/crc_case.py ${STRIDE:-320} ${LEN:-312} ${N:-10000000} 1024 1048576 3 > /dev/null 2>&1 || exit $?
  done
done
