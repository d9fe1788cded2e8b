#!/bin/bash
# Build the libavt.so of a git revision (default HEAD) as audio-visual-tubes_amd/libavt_base.so, for same-box
# A/B runs (AVT_LIB_PATH=.../libavt_base.so).  usage: bash tools/build_base.sh [rev]
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/avt_base_XXXX)
git -C "$R" worktree add -q --detach "$W" "$REV"
cd "$W/audio-visual-tubes_amd/csrc"
objs=""
for f in conv_gemm bn pool head misc tube eval audio frames; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$W/include" -c $f.hip -o $W/$f.o &
  objs="$objs $W/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o "$R/audio-visual-tubes_amd/libavt_base.so" $objs
git -C "$R" worktree remove --force "$W"
echo "built $R/audio-visual-tubes_amd/libavt_base.so from $(git -C "$R" rev-parse --short $REV)"
