# team-size A/B over record lengths: G=1 policy, G=2, G=16/64
TAG=g1 timeout -k 10 200 python3 tools/team_sweep.py > gpurun_out/ts_g1.log 2>&1 &&
TAG=g2 ZSCRC_SMALL_TEAM=2 timeout -k 10 200 python3 tools/team_sweep.py > gpurun_out/ts_g2.log 2>&1 &&
TAG=g16 ZSCRC_G1_MAX=0 timeout -k 10 200 python3 tools/team_sweep.py > gpurun_out/ts_g16.log 2>&1
