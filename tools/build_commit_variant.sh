# Build gym_po_amd/libgympo_amd_<NAME>.so from the csrc/ + include/ of git commit <COMMIT> (every source), for
# in-call A/B runs of kernel versions (GYM_PO_AMD_LIB=.../libgympo_amd_<NAME>.so; tools/gpu.sh ab "NAME ...").
#   bash tools/build_commit_variant.sh NAME COMMIT
set -e
NAME=$1
COMMIT=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/gym-po-taxi_amd/build/cvar_$NAME
rm -rf $D && mkdir -p $D/obj
(cd $ROOT && git archive $COMMIT gym-po-taxi_amd/csrc include) | tar -x -C $D
for f in $D/gym-po-taxi_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -O3 -Wno-unused-result -I $D/include \
    -c $f -o $D/obj/$(basename ${f%.hip}).o 2>/dev/null &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/gym-po-taxi_amd/gym_po_amd/libgympo_amd_$NAME.so $D/obj/*.o
echo "built libgympo_amd_$NAME.so from $COMMIT"
