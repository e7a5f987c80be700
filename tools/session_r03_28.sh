# dynamic-unit qteam: tail probe, parity, A/B, wave timing; then the final-build checks
O=gpurun_out/trace_bench
bash tools/gpu_session.sh \
 "tail:200:./tools/tail_probe" \
 "t_q:500:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'qteam or headline'" \
 "abq:300:AB_CASES=config3,fixed_16KiB,fixed_4KiB python tools/opt_ab.py 0 32" \
 "abqP:300:ZSCRC_QDYN_P=8 AB_CASES=config3 python tools/opt_ab.py 0 32" \
 "waves:300:WAVES_C3=1 python tools/xparts_waves.py" \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench3:300:python bench.py"
