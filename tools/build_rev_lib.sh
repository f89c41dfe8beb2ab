# Build libgympo_amd.so of git revision $1 into gym-po-taxi_amd/gym_po_amd/libgympo_amd_${2:-ab}.so (for in-call
# A/B runs with GYM_PO_AMD_LIB pointing at it). Uses a temporary git worktree.
set -e
REV=${1:-HEAD~1}
NAME=${2:-ab}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/gp_wt.XXXX)
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
python "$WT/gym-po-taxi_amd/build.py" --force > /dev/null
cp "$WT/gym-po-taxi_amd/gym_po_amd/libgympo_amd.so" "$ROOT/gym-po-taxi_amd/gym_po_amd/libgympo_amd_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $REV -> gym-po-taxi_amd/gym_po_amd/libgympo_amd_$NAME.so"
