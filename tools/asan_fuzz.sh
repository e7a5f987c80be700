#!/bin/bash
# AddressSanitizer + UBSan campaign over libzscrc's host-side zeroskip parsers
# (tests/c/parse_fuzz.c): the host objects of the library rebuilt with
# -fsanitize=address,undefined (clang throughout; the device code as usual,
# GPU sanitizers are not used), linked into the fuzzer, run on the CPU over
# mutated copies of the reference-written fixtures.  No GPU is touched.
# usage: bash tools/asan_fuzz.sh [ITERATIONS] [SEEDS...]   (outputs under /tmp/zs_asan)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/zs_asan
N=${1:-10000}; shift || true
SEEDS=${*:-"11 12 13 14"}
CL=/opt/rocm/llvm/bin/clang
RT=$(dirname "$(find /opt/rocm/llvm/lib/clang -name 'libclang_rt.asan-x86_64.so' | head -1)")
rm -rf $W && mkdir -p $W/zeroskip_amd && cp -r "$R/zeroskip_amd/csrc" "$R/zeroskip_amd/Makefile" $W/zeroskip_amd/ && cp -r "$R/include" $W/
SAN="-fsanitize=address -fsanitize=undefined -fno-omit-frame-pointer -g"
OBJS="build/zscrc_kernels.o build/zscrc_api.o build/zscrc_zs.o build/zscrc_consistent.o build/zscrc_gf2.o \
      build/zscrc_cpu.o build/zscrc_pack.o build/zscrc_files.o build/zscrc_repack.o build/zscrc_cpass.o build/zscrc_fill.o"
( cd $W/zeroskip_amd && make -s -j8 \
    HIPFLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer" \
    CC="$CL" CFLAGS="-O1 -fPIC -std=gnu11 $SAN" CXX="${CL}++ $SAN" $OBJS && \
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -shared-libasan -o libzscrc.so $OBJS -lpthread )
$CL -O1 $SAN -I"$R/include" "$R/tests/c/parse_fuzz.c" -L$W/zeroskip_amd -lzscrc -Wl,-rpath,$W/zeroskip_amd \
    -shared-libasan -o $W/parse_fuzz
python3 -c "import sys; sys.path.insert(0, '$R'); from oracle import zs_format as zf; \
open('$W/dotzsdb', 'wb').write(zf.dotzsdb_bytes(4096, b'00010203-0405-0607-0809-0a0b0c0d0e0f\0', 8))"
F=$R/tests/golden/ref_format
for s in $SEEDS; do
  LD_LIBRARY_PATH=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 ZSCRC_GPU_MIN=0 $W/parse_fuzz "$N" "$s" \
    $F/active_clean.zs $F/active_corrupt.zs $F/active_stale.zs $F/active_longkey.zs $F/packed.zs \
    $F/repack1/reference_out.zs $F/repack2/reference_out.zs $W/dotzsdb
done
