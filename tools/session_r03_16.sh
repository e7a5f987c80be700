# parity after the multi64 / xteam scheduling fixes; A/B of the pins (opt 128 / 512) and of the
# branch-free xteam issue (library A/B); the in-place store probe with 128 B lines and plain loads
bash tools/gpu_session.sh \
 "t_par:400:python -u -m pytest tests/test_gpu_longspans.py tests/test_gpu_parity.py tests/test_gpu_zsfile.py tests/test_gpu_consistent.py tests/test_gpu_files.py -x -q --timeout 120 --timeout-method thread" \
 "abpin:300:AB_CASES=config2_multi32,config4_nb,fixed_1MiB,span_3GiB python tools/opt_ab.py 0 128 512" \
 "abflat:400:bash tools/lib_ab.sh tools/ab/libzscrc_noflat.so config4_nb,fixed_1MiB,span_3GiB" \
 "runprobe:200:./tools/run_probe"
