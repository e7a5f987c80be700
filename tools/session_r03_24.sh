# qteam / xteam on 2x / 4x grids (block-level balancing of the tail), interleaved A/B
bash tools/gpu_session.sh \
 "abgrid:400:AB_CASES=config3,fixed_1MiB,config4_verdict python tools/opt_ab.py 0 32 64"
