#!/bin/bash
# Build a whole-library A/B variant (every source recompiled with extra -D flags, e.g. a header
# switch such as -DXS_F32=0): abl/libcsm_hip_<name>.so.  usage: tools/fullvariant.sh <name> <flags...>
set -e
name=$1; shift
cd "$(dirname "$0")/.."
b=/tmp/fv_$name; mkdir -p $b abl
for src in csm-mlx_amd/csrc/*.hip csm-mlx_amd/csrc/*.cpp; do
  f=$(basename $src); extra=""
  case $f in dec_frame.hip|bb_step.hip) extra="-mllvm -amdgpu-use-amdgpu-trackers=1";; esac
  lang=""; case $f in *.hip) lang="-x hip";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $extra "$@" -Icsm-mlx_amd/csrc $lang -c $src -o $b/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libcsm_hip_$name.so $b/*.o
echo abl/libcsm_hip_$name.so
