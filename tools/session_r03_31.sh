# TA address-stall ratio of the bare run-round shapes (tools/run_probe.hip) and the streaming read
# (tools/tail_probe.hip static) beside commit_kernel's 0.54: is the stall the address path or HBM back-pressure?
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES --output-format csv -d $R/gpurun_out/pmc_runprobe -o run -- $R/tools/run_probe > $R/gpurun_out/pmc_runprobe.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES --output-format csv -d $R/gpurun_out/pmc_tail -o run -- $R/tools/tail_probe > $R/gpurun_out/pmc_tail.log 2>&1
