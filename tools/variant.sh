#!/bin/bash
# Build an A/B variant of libcsm_hip.so: one source recompiled with extra -D flags, linked with the
# current in-tree objects.  usage: tools/variant.sh <name> <source.hip> <flags...>  -> lab/libcsm_hip_<name>.so
# (run with CSM_HIP_LIB=$PWD/lab/libcsm_hip_<name>.so).  VARIANT_FILE=<path> compiles that file in
# place of csrc/<source.hip> (e.g. an older revision from git show).
set -e
name=$1; src=$2; shift 2
OUT=${VARIANT_DIR:-lab}  # not gpurun-ignored: the variant travels to the GPU box (abl/ does not)
cd "$(dirname "$0")/.."
python -c "import __graft_entry__ as g; g.build()" > /dev/null
mkdir -p $OUT
b=csm-mlx_amd/build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -Icsm-mlx_amd/csrc -x hip -c ${VARIANT_FILE:-csm-mlx_amd/csrc/$src} -o /tmp/variant_$name.o
objs=$(ls $b/*.o | grep -v "/$src.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libcsm_hip_$name.so $objs /tmp/variant_$name.o
echo $OUT/libcsm_hip_$name.so
