# Build gym_po_amd/libgympo_amd_<NAME>.so with extra compile flags on grid.hip (other sources: the release
# objects), for in-call A/B runs (GYM_PO_AMD_LIB=.../libgympo_amd_<NAME>.so).
#   bash tools/build_variant.sh NAME "-DFOO=1 -DBAR=0"
set -e
NAME=$1
FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/gym-po-taxi_amd/build/var_$NAME
mkdir -p $OBJ
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -O3 -Wno-unused-result $FLAGS -I $ROOT/include \
  -c $ROOT/gym-po-taxi_amd/csrc/grid.hip -o $OBJ/grid.o
R=$ROOT/gym-po-taxi_amd/build/${BASE:-release}  # BASE=stamps for GP_STAMPS variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/gym-po-taxi_amd/gym_po_amd/libgympo_amd_$NAME.so \
  $R/anttag.o $R/api.o $R/crooms.o $R/dist.o $OBJ/grid.o $R/taxi.o
echo "built libgympo_amd_$NAME.so ($FLAGS)"
