#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# Build the working tree's library with extra hipcc flags into
# go_raytracer_amd/build_abl/NAME/librt_amd.so (dev tool, A/B variants):
#   tools/build_variant.sh NAME "-DMESH_WLDS=2 -DMESH_SHORT=12"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2
mkdir -p "$R/go_raytracer_amd/build_abl/$NAME"
rm -rf "/tmp/rt_var_$NAME"  # make does not track FLAGS: always a fresh build
make -s -C "$R/go_raytracer_amd/csrc" -j8 OUT="$R/go_raytracer_amd/build_abl/$NAME/librt_amd.so" \
  BUILD="/tmp/rt_var_$NAME" EXTRA_HIPFLAGS="$FLAGS" "$R/go_raytracer_amd/build_abl/$NAME/librt_amd.so"
ls -la "$R/go_raytracer_amd/build_abl/$NAME/librt_amd.so"
