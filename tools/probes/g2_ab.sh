# A/B of the record-burst kernels: plain per-lane loads vs ZS_BURST_XP (quad-cooperative loads + permlane transpose)
timeout -k 10 200 python3 tools/probes/g1_sweep.py > gpurun_out/ga.log 2>&1 &&
ZS_BURST_XP=1 timeout -k 10 200 python3 tools/probes/g1_sweep.py > gpurun_out/gb.log 2>&1
