#!/bin/bash
# Per-instantiation VGPRs / scratch bytes per lane of a HIP source: tools/resource_usage.sh [file.hip]
F=${1:-learning-based-mpc_amd/csrc/bqp_ocp.hip}
/opt/rocm/bin/hipcc $EXTRA -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-result -Wno-unused-value -x hip -c "$F" -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | \
  python3 -c "
import re,sys
cur=None; v={}
for ln in sys.stdin:
    m=re.search(r'Function Name: (\S+)',ln)
    if m: cur=m.group(1); v[cur]=['?','?']; continue
    m=re.search(r' VGPRs: (\d+)',ln)
    if m and cur: v[cur][0]=m.group(1)
    m=re.search(r'ScratchSize \[bytes/lane\]: (\d+)',ln)
    if m and cur: v[cur][1]=m.group(1)
for k,(a,b) in v.items():
    m=re.search(r'ocp_ipm_kernelI((?:Li\d+E)+)',k)
    name='ocp<'+','.join(re.findall(r'Li(\d+)E',m.group(1)))+'>' if m else k[:60]
    print('%-40s vgpr %4s scratch %5s'%(name,a,b))
"
