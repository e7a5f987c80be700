bash tools/gpu_session.sh \
 "tail:200:./tools/tail_probe" \
 "t_q:300:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'qteam_shapes'" \
 "abq:300:AB_CASES=config3 python tools/opt_ab.py 0 32" \
 "abq64:300:ZSCRC_QDYN_P=64 AB_CASES=config3 python tools/opt_ab.py 0 32"
