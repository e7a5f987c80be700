# L2->memory read requests by size for short-record layouts and the probe.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/rdreq; mkdir -p $O
P="TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum"
for c in fixed64_64_0 fixed320_320_0 fixed320_312_40; do
  timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/$c -o run -- python3 $R/tools/prof_case.py $c 5 > $O/$c.log 2>&1 || exit $?
done
timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/probe -o run -- $R/tools/probes/short_probe > $O/probe.log 2>&1 || exit $?
