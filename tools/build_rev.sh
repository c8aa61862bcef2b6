# Build libramcrc from the sources of a git revision into
# ramcloud_amd/lib/variants/libramcrc_<name>.so (A/B of the working tree
# against a committed state).
#   bash tools/build_rev.sh HEAD head
set -e
REV=$1
NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" ramcloud_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$ROOT/ramcloud_amd/lib/variants"
cd "$TMP"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fconstexpr-steps=1000000000 \
    -Iinclude -Iramcloud_amd/csrc -DRAMCRC_SRC_SHA="\"rev-$NAME\"" \
    ramcloud_amd/csrc/ramcrc_device.hip ramcloud_amd/csrc/ramcrc_host.cc \
    ramcloud_amd/csrc/ramcrc_shard.hip ramcloud_amd/csrc/ramcrc_fill.hip -ldl \
    -o "$ROOT/ramcloud_amd/lib/variants/libramcrc_$NAME.so"
rm -rf "$TMP"
echo "$ROOT/ramcloud_amd/lib/variants/libramcrc_$NAME.so"
