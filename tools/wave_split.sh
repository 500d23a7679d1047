#!/bin/bash
# Resource usage of the MG C2 kernel with only the stage wave / only the row wave compiled
# (codegen inspection; never built into the product).  usage: tools/wave_split.sh
cd "$(dirname "$0")/../learning-based-mpc_amd"
for M in BQP_XX_STAGE BQP_XX_ROW; do
  sed -e "s/    if (!rowwave)\$/#ifdef BQP_XX_ROW\n    if (0)\n#else\n    if (!rowwave)\n#endif/" \
      -e "s/^    else\$/#ifdef BQP_XX_STAGE\n    else if (0)\n#else\n    else\n#endif/" csrc/bqp_ocp.hip > /tmp/ocp_$M.hip
  echo "== $M"
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -I csrc -I ../include -D$M -DBQP_ISA_ONLY_MG10 \
    -x hip -S --cuda-device-only /tmp/ocp_$M.hip -o /tmp/ocp_$M.s -Rpass-analysis=kernel-resource-usage 2>&1 \
    | grep -E "VGPRs:|Scratch|VGPRs Spill" | sed 's/.*remark: *//; s/ \[-R.*//'
  python ../tools/isa_loops.py /tmp/ocp_$M.s | sort -k4 -n -r | head -1
done
