#!/bin/bash
# kernel_regs.sh [EXTRA flags] -- per-kernel VGPR / AGPR / SGPR / LDS /
# scratch of the gfx950 K2 translation unit, as the compiler reports them
# (-Rpass-analysis=kernel-resource-usage).  EXTRA=-DRF_DIAG: the diagnostic build.
cd "$(dirname "$0")/../reflow_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include ${EXTRA} \
    --offload-device-only -c ${SRC:-k2_graph.hip} -o /tmp/kregs.$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c '
import sys, re
cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur: rows[cur][m.group(1).split()[0].replace("Total", "")] = m.group(2)
for k, v in rows.items():
    print("%-70s VGPR %4s AGPR %3s SGPR %3s scratch %4s LDS %6s occ %s" % (k[:70], v.get("VGPRs"), v.get("AGPRs"), v.get("SGPRs"), v.get("ScratchSize"), v.get("LDS"), v.get("Occupancy")))
'
rm -f /tmp/kregs.$$.o
