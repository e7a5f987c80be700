bash tools/gpu_session.sh \
 "trace:900:bash tools/trace_bench.sh config4 config5 config2 config3" \
 "pmc4:200:bash tools/pmc_case.sh config4" \
 "tr4:200:bash tools/pmc_traffic.sh config4" \
 "tr5:200:bash tools/pmc_traffic.sh config5" \
 "pmc4w:200:bash tools/pmc_case.sh config4w" \
 "tr4w:200:bash tools/pmc_traffic.sh config4w"
