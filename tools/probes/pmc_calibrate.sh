# FETCH_SIZE / L2 request+miss counts of tools/prof_case.py fixed-stride layouts
# per short-kernel walk (ZS_DEPTH), plus their timings (tools/probes/g1_sweep-like).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/cal; mkdir -p $O
for c in ${CASES:-fixed320_312_40 fixed320_320_0 fixed64_64_0}; do
 for dp in ${DEPTHS:-3 9}; do
  ZS_DEPTH=$dp timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${c}_d${dp}_fetch -o run -- python3 $R/tools/prof_case.py $c 5 > $O/${c}_d${dp}.log 2>&1 || exit $?
  ZS_DEPTH=$dp timeout -s KILL 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/${c}_d${dp}_tcc -o run -- python3 $R/tools/prof_case.py $c 5 >> $O/${c}_d${dp}.log 2>&1 || exit $?
  ZS_DEPTH=$dp timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/${c}_d${dp}_trace -o run -- python3 $R/tools/prof_case.py $c 5 >> $O/${c}_d${dp}.log 2>&1 || exit $?
 done
done
