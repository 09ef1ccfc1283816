#!/bin/bash
# Analysis builds of the LDS-DMA weight gradient (CPU side, repo root): conv.hip compiled with
# -DWG_CUT=1 (no operand DMA inside the loop) and -DWG_CUT=2 (no MFMAs), linked with the other
# objects of csrc/_build into _scratch/_C_cut{1,2}.so.  On the GPU box:
#   python tools/wgrad_cut.py 1 <wgrad_probe args>   (loads _scratch/_C_cut1.so instead of _C.so)
set -e
mkdir -p _scratch
objs=$(ls simclr_amd/csrc/_build/*.o | grep -v '/conv.o$')
libs=$(python -c "import torch.utils.cpp_extension as ce; print(' '.join('-L'+d+' -Wl,-rpath,'+d for d in ce.library_paths()))")
for c in 1 2; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -std=c++17 -O3 -Wno-unused-result -DWG_CUT=$c \
    -c simclr_amd/csrc/conv.hip -o _scratch/conv_cut$c.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o _scratch/_C_cut$c.so \
    _scratch/conv_cut$c.o $objs $libs -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip
done
