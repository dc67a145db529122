# Build the library of a git revision (default HEAD) as the A/B baseline
# superresolution_for_pdes_amd/lib/ab/libsrpde_hip_base.so (SRPDE_LIB selects it at run time).
#   bash tools/build_base.sh [REV]
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/srpde_base_$$
git -C "$ROOT" worktree add -f --detach "$W" "$REV" > /dev/null
(cd "$W" && SRPDE_BUILD_OUT="$ROOT/superresolution_for_pdes_amd/lib/ab/libsrpde_hip_base.so" python -m superresolution_for_pdes_amd.build --force)
git -C "$ROOT" worktree remove --force "$W"
ls -la "$ROOT/superresolution_for_pdes_amd/lib/ab/libsrpde_hip_base.so"
