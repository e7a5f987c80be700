# The in-place writer's whole-64-byte-block stores, measured in the product's
# own loop: a second libzscrc built with
# -DZS_DIAG_BLOCK_STORE=1 (emit stores the aligned 64-byte block around each
# CRC field, filled with the CRC -- wrong image bytes, timing only) against
# the shipped build, interleaved over three rounds; =2 also reads the run
# rounds with non-temporal loads (the writer's plain loads keep the line of a
# 4-byte store in the L2; a whole-block store does not need it there).
# Build (CPU, in-tree so it travels): bash tools/probes/block_store_ab.sh build
# Run (GPU box):                      bash tools/probes/block_store_ab.sh run
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
if [ "$1" = build ]; then
  mkdir -p /tmp/zs_diag
  H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall"
  objs=$(ls zeroskip_amd/build/*.o | grep -v zscrc_kernels.o)
  for v in 1 2; do
    $H -DZS_DIAG_BLOCK_STORE=$v -c zeroskip_amd/csrc/zscrc_kernels.hip -o /tmp/zs_diag/zscrc_kernels$v.o
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o zeroskip_amd/libzscrc_diagblock$v.so \
      /tmp/zs_diag/zscrc_kernels$v.o $objs -lpthread
  done
  exit 0
fi
AB_OUT=${AB_OUT:-gpurun_out/r06/block_store_ab.log}
mkdir -p "$(dirname "$AB_OUT")"
: > "$AB_OUT"
for v in 1 2; do
  ZSCRC_LIB_PATH=zeroskip_amd/libzscrc_diagblock$v.so timeout -k 10 120 python tools/probes/block_store_check.py \
    >> "$AB_OUT" 2>&1
done
for r in 1 2 3; do
  for L in zeroskip_amd/libzscrc.so zeroskip_amd/libzscrc_diagblock1.so zeroskip_amd/libzscrc_diagblock2.so; do
    echo "round $r: $L" >> "$AB_OUT"
    ZSCRC_LIB_PATH=$L AB_CASES=config4_write timeout -k 10 200 python tools/opt_ab.py 0 >> "$AB_OUT" 2>&1
  done
done
