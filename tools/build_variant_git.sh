# Build an A/B variant of the library with ONE source file taken from a git revision (the other objects are
# reused from superresolution_for_pdes_amd/lib/obj):   bash tools/build_variant_git.sh OUT.so REV SOURCE.hip [SED_EXPR]
# REV "WORKTREE" takes the working copy; SED_EXPR (optional) is applied to the source first (a one-line A/B switch).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; REV=$2; SRC=$3; SEDX=${4:-}
OBJ=$ROOT/superresolution_for_pdes_amd/lib/obj
TMPS=$ROOT/superresolution_for_pdes_amd/csrc/.variant_$SRC
TMPO=$(mktemp /tmp/variant_XXXX.o)
if [ "$REV" = WORKTREE ]; then cp $ROOT/superresolution_for_pdes_amd/csrc/$SRC $TMPS; else git -C $ROOT show $REV:superresolution_for_pdes_amd/csrc/$SRC > $TMPS; fi
if [ -n "$SEDX" ]; then sed -i "$SEDX" $TMPS; fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -Xclang -target-feature -Xclang -packed-fp32-ops -x hip -c $TMPS -o $TMPO 2>/dev/null
rm -f $TMPS
OBJS=$(ls $OBJ/*.o | grep -v "/$SRC.o")
mkdir -p $(dirname $OUT)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $OBJS $TMPO
rm -f $TMPO
echo $OUT
