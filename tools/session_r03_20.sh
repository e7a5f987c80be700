# segment plans for class 3: parity (long spans, runs, consistent, files), A/B against per-record parts,
# per-wave timing
bash tools/gpu_session.sh \
 "t_long:400:python -u -m pytest tests/test_gpu_longspans.py tests/test_gpu_parity.py tests/test_gpu_consistent.py tests/test_gpu_files.py tests/test_gpu_zsfile.py -x -q --timeout 120 --timeout-method thread" \
 "abseg:300:AB_CASES=config4_nb python tools/opt_ab.py 0 256" \
 "waves:300:python tools/xparts_waves.py"
