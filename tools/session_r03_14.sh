# SQ instruction / wait / LDS counters for config 2 (multi64_kernel) beside config 3 (qteam_kernel);
# kernel trace of the NOTBATCHED verdict pass sequence
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/nbtrace -o run -- python3 $R/tools/prof_case.py config4nb 20 > $R/gpurun_out/nbtrace.log 2>&1) && \
python tools/seq_trace.py gpurun_out/nbtrace 2 > gpurun_out/nbseq.txt && \
bash tools/gpu_session.sh \
 "pmc2:400:bash tools/pmc_case.sh config2" \
 "pmc3:400:bash tools/pmc_case.sh config3"
