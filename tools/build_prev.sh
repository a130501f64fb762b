#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# Build the library of git revision REV (default HEAD) into go_raytracer_amd/build_prev (A/B baseline).
REV=${1:-HEAD}
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
rm -rf /tmp/rt_prev && mkdir -p /tmp/rt_prev "$R/go_raytracer_amd/build_prev"
git -C "$R" archive "$REV" go_raytracer_amd/csrc include | tar -x -C /tmp/rt_prev
make -s -C /tmp/rt_prev/go_raytracer_amd/csrc -j8 ROOT=/tmp/rt_prev \
  OUT="$R/go_raytracer_amd/build_prev/librt_amd.so" BUILD=/tmp/rt_prev/build 2>&1 | grep -E "error" || true
ls -la "$R/go_raytracer_amd/build_prev/librt_amd.so"
