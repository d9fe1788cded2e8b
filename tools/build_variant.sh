#!/bin/bash
# Build the WORKING TREE's libavt with extra compiler flags as audio-visual-tubes_amd/<name>, for same-box
# A/B runs (AVT_LIB_PATH=...).  usage: bash tools/build_variant.sh libavt_base.so -DAVT_BN_SLOTS=16
set -e
NAME=$1; shift
[ "$NAME" = libavt.so ] && { echo "build libavt.so with __graft_entry__.build() (it records the source hash)"; exit 2; }
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/avt_var_XXXX)
objs=""
for f in conv_gemm bn pool head misc tube eval audio frames; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/include" "$@" -c "$R/audio-visual-tubes_amd/csrc/$f.hip" -o $W/$f.o &
  objs="$objs $W/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o "$R/audio-visual-tubes_amd/$NAME" $objs
rm -rf "$W"
echo "built $R/audio-visual-tubes_amd/$NAME with $*"
