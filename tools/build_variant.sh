#!/bin/bash
# build_variant.sh NAME "EXTRA HIPCC FLAGS" -> tools/ab/NAME.so
# (built with -DRTMI_DIAG: the RTMI_* diagnostic / A/B environment knobs are
# read only by such builds, rt_common.h diag_env)
# (the kernel TUs — float32 main + the 16 specialisation parts, the float64
# kernels, the per-call build and the host launch code — and every TU that
# reads a diag_env knob (rt_bins.cpp: RTMI_GRID_DENSITY, rt_bvh_gpu.hip:
# RTMI_PLOC_RADIUS) rebuilt with the flags; ADVICE r5: linking the normal
# rt_bins.o made the density knob a no-op in diagnostic builds)
set -e
cd "$(dirname "$0")/../nim-raytracer_amd"
set -- "$1" "-DRTMI_DIAG $2"
make -s -j8 >/dev/null
mkdir -p ../tools/ab build/var/$1
F="-O3 -std=c++17 -fPIC ${F32_FLAGS--ffp-contract=fast -Xclang -target-feature -Xclang -packed-fp32-ops -mllvm -amdgpu-atomic-optimizer-strategy=None} $2"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c csrc/rt_kernels_f32.hip -o build/var/$1/main.o 2> >(grep -v "packed-fp32-ops. is not a recognized" >&2) &
for k in $(seq 0 15); do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -DRTMI_PART=$k -c csrc/rt_kernels_f32_part.hip -o build/var/$1/part$k.o 2> >(grep -v "packed-fp32-ops. is not a recognized" >&2) &
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $2 -c csrc/rt_frame.hip -o build/var/$1/frame.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $2 -c csrc/rt_kernels_f64.hip -o build/var/$1/f64.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=off $2 -c csrc/rtmi.cpp -o build/var/$1/rtmi.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=off $2 -c csrc/rt_bins.cpp -o build/var/$1/bins.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=off $2 -c csrc/rt_bvh_gpu.hip -o build/var/$1/bvh_gpu.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/ab/$1.so build/var/$1/main.o build/var/$1/part*.o build/var/$1/f64.o build/rt_kernels_io.o build/var/$1/rtmi.o build/rt_bvh.o build/var/$1/bvh_gpu.o build/rt_queue.o build/rt_obj.o build/rt_multi.o build/var/$1/bins.o build/var/$1/frame.o
