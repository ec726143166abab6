#!/bin/bash
# Build A/B variants of libcista_hip.so into v2e2v_amd/variants/<name>.so: the same sources with
# extra -D switches (timing: scripts/ab_layers.sh on the GPU box; parity of every variant:
# `bash scripts/gpu_check.sh vtests`).  The in-tree default build is not touched.
# usage: bash scripts/build_variants.sh name1 "-DFLAG=1 ..." [name2 "-D..." ...]
set -e
cd "$(dirname "$0")/.."
make -s build/cista_ssim.o build/cista_v2e.o
mkdir -p build/variants v2e2v_amd/variants
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  (
    $HIPCC -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result $flags \
      -c -o build/variants/$name.o v2e2v_amd/csrc/cista_abi.hip &&
    $HIPCC -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result $flags \
      -c -o build/variants/${name}_vox.o v2e2v_amd/csrc/cista_voxel.hip &&
    $HIPCC --offload-arch=gfx950 -shared -o v2e2v_amd/variants/$name.so build/variants/$name.o \
      build/variants/${name}_vox.o build/cista_ssim.o build/cista_v2e.o && echo "built $name ($flags)"
  ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
