# VGPR / spill / occupancy of the engine's own kernels in one HIP source (diagnostics)
# usage: bash tools/vgprs.sh sentinel_amd/csrc/sf_kernels.hip
SRC=${1:-sentinel_amd/csrc/sf_kernels.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -c -x hip $SRC -o /tmp/vg.o \
  -Rpass-analysis=kernel-resource-usage $EXTRA 2>&1 | python3 -c "
import sys,re
name=None
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: name=m.group(1); continue
    if name and 'rocprim' in name: continue
    for k in ('VGPRs:','AGPRs:','ScratchSize','Occupancy'):
        if k in l and name: print(name[:60], l.split('remark: ')[-1].strip())
"
