#!/bin/bash
# Build engine variants for A/B timing: tools/build_variants.sh name1="-DFOO" name2="-DBAR -DBAZ" ...
# -> build/ab/<name>/libartis_gpu.so (git-ignored; travels to the GPU box), loaded with ARTIS_GPU_SO=<path>.
cd "$(dirname "$0")/.."
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  mkdir -p build/ab/$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared $flags -Iinclude \
    -Iartis_amd/csrc/engine artis_amd/csrc/engine/engine.hip -o build/ab/$name/libartis_gpu.so -L/opt/rocm/lib -lrccl \
    -Wl,-rpath,/opt/rocm/lib > build/ab/$name/build.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
