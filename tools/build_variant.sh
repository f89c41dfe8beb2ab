# Build gym_po_amd/libgympo_amd_<NAME>.so with extra compile flags on some sources (default: wgrid.hip and
# grid.hip, which share grid_shared.h; the other sources: the release objects), for in-call A/B runs
# (GYM_PO_AMD_LIB=.../libgympo_amd_<NAME>.so).
#   bash tools/build_variant.sh NAME "-DFOO=1 -DBAR=0" ["a.hip b.hip"]
set -e
NAME=$1
FLAGS=$2
SRCS=${3:-wgrid.hip grid.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/gym-po-taxi_amd/build/var_$NAME
mkdir -p $OBJ
R=$(ls -d $ROOT/gym-po-taxi_amd/build/${BASE:-release}-* | head -1)  # BASE=stamps for GP_STAMPS variants
EXTRA=""
[ "${BASE:-release}" = stamps ] && EXTRA="-DGP_STAMPS"
for S in $SRCS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -O3 -Wno-unused-result $EXTRA $FLAGS -I $ROOT/include \
    -c $ROOT/gym-po-taxi_amd/csrc/$S -o $OBJ/${S%.hip}.o &
done
wait
OBJS=""
for o in $R/*.o; do
  case " $SRCS " in *" $(basename ${o%.o}).hip "*) continue ;; esac
  OBJS="$OBJS $o"
done
for S in $SRCS; do OBJS="$OBJS $OBJ/${S%.hip}.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/gym-po-taxi_amd/gym_po_amd/libgympo_amd_$NAME.so $OBJS
echo "built libgympo_amd_$NAME.so ($SRCS $FLAGS)"
