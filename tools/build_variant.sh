#!/bin/bash
# build_variant.sh NAME "EXTRA HIPCC FLAGS" -> tools/ab/NAME.so (f32 kernel TU rebuilt with the flags)
set -e
cd "$(dirname "$0")/../nim-raytracer_amd"
make -s -j4 >/dev/null
mkdir -p ../tools/ab build/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC ${F32_FLAGS--ffp-contract=fast -Xclang -target-feature -Xclang -packed-fp32-ops} $2 -c csrc/rt_kernels_f32.hip -o build/var/$1.o 2> >(grep -v "packed-fp32-ops. is not a recognized" >&2)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/ab/$1.so build/var/$1.o build/rt_kernels_f64.o build/rtmi.o build/rt_bvh.o
