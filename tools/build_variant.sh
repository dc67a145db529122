# Build an A/B variant of the library that differs from the in-tree build in ONE source file's compile
# flags (the other objects are reused from superresolution_for_pdes_amd/lib/obj):
#   bash tools/build_variant.sh OUT.so SOURCE.hip [extra hipcc flags...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; SRC=$2; shift 2
OBJ=$ROOT/superresolution_for_pdes_amd/lib/obj
TMPO=$(mktemp /tmp/variant_XXXX.o)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -Xclang -target-feature -Xclang -packed-fp32-ops "$@" -c $ROOT/superresolution_for_pdes_amd/csrc/$SRC -o $TMPO 2>/dev/null
OBJS=$(ls $OBJ/*.o | grep -v "/$SRC.o")
mkdir -p $(dirname $OUT)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $OBJS $TMPO
rm -f $TMPO
echo $OUT
