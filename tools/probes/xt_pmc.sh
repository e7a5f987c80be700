# PMC comparison of xteam on 64 KiB vs 1 MiB records (4 GiB each)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/xtpmc
mkdir -p $O
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY"
for case in "65536 65536" "1048576 4096"; do
  set -- $case
  for k in 1 2; do
    eval C=\$C$k
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/L$1_p$k -o run -- python3 $R/tools/probes/xt_prof.py $1 $2 1 > $O/L$1_p$k.log 2>&1 || exit $?
  done
done
