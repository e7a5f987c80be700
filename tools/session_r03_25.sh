# where commit_kernel's time goes: diagnostics without the chains (4096) / without the trailer + stores (8192)
bash tools/gpu_session.sh \
 "abc4:400:AB_CASES=config4_verdict,config4_verify python tools/opt_ab.py 0 4096 8192 12288"
