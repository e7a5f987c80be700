# dynamic-unit qteam: parity (config 3 full size, ragged shapes, P variants), interleaved A/B, wave timing
bash tools/gpu_session.sh \
 "t_q:500:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'qteam or headline'" \
 "abq:300:AB_CASES=config3,fixed_16KiB,fixed_4KiB python tools/opt_ab.py 0 32" \
 "abqP:300:ZSCRC_QDYN_P=8 AB_CASES=config3 python tools/opt_ab.py 0 32" \
 "waves:300:WAVES_C3=1 python tools/xparts_waves.py"
