# Kernel sequences of config 4 NOTBATCHED's three forms (ranged verdict,
# unranged verdict, per-commit arrays), one rocprofv3 kernel trace each.
# usage (GPU box): bash tools/probes/nb_seq.sh
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/nbseq
mkdir -p $O
for m in range unranged arrays; do
  C4NB_MODE=$m timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o run -- \
      python3 $R/tools/prof_case.py config4nb 10 > $O/$m.log 2>&1 || exit $?
  python3 $R/tools/probes/seq_trace.py $O/$m 3 > $O/$m.txt 2>&1 || exit $?
done
