# A/B: multi64 walk order / nt stores (config 2), balanced xteam parts (NOTBATCHED); parity of both paths
bash tools/gpu_session.sh \
 "t_par:300:python -u -m pytest tests/test_gpu_longspans.py tests/test_gpu_parity.py tests/test_gpu_zsfile.py -x -q --timeout 120 --timeout-method thread" \
 "ab2:300:AB_CASES=config2_multi32,config2_warm32 python tools/opt_ab.py 0 32 64 96" \
 "abnb:300:AB_CASES=config4_nb python tools/opt_ab.py 0 256 131072 131328"
