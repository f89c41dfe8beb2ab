# Like build_variant.sh for any one source: bash tools/build_variant_src.sh NAME SRC.hip "FLAGS"
set -e
NAME=$1; SRC=$2; FLAGS=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/gym-po-taxi_amd/build/var_$NAME
mkdir -p $OBJ
R=$ROOT/gym-po-taxi_amd/build/${BASE:-release}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -O3 -Wno-unused-result $FLAGS -I $ROOT/include \
  -c $ROOT/gym-po-taxi_amd/csrc/$SRC -o $OBJ/${SRC%.hip}.o
objs=""
for f in $R/*.o; do b=$(basename $f); if [ "$b" = "${SRC%.hip}.o" ]; then objs="$objs $OBJ/$b"; else objs="$objs $f"; fi; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/gym-po-taxi_amd/gym_po_amd/libgympo_amd_$NAME.so $objs
echo "built libgympo_amd_$NAME.so ($SRC $FLAGS)"
