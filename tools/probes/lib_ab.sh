# A/B of two libzscrc builds: tools/opt_ab.py runs alternately with each (3 rounds)
# usage: bash tools/probes/lib_ab.sh <other.so> [cases]
OTHER=$1
CASES=${2:-config3,config4_verify,config2_multi32,config2_warm32,fixed_320x312}
for r in 1 2 3; do
  echo "round $r: default build"
  AB_CASES=$CASES timeout -k 10 200 python tools/opt_ab.py 0 || exit $?
  echo "round $r: $OTHER"
  ZSCRC_LIB_PATH=$OTHER AB_CASES=$CASES timeout -k 10 200 python tools/opt_ab.py 0 || exit $?
done
