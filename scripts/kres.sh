#!/bin/bash
# Register / LDS / scratch use of the kernels of one source (hipcc remarks).
# Usage: scripts/kres.sh SRC(e.g. gf) [kernel-substring] [extra hipcc flags...]
S=$1; K=${2:-.}; shift 2
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-function --cuda-device-only -c "$@" \
  gf_orb_slam_amd/csrc/$S.hip -o /tmp/kres_$S.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed 's/.*remark: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk -v k="$K" '/Function Name:/ {name=$3; show=(name ~ k)} show && /VGPRs:|AGPRs:|ScratchSize|Occupancy|LDS Size|SGPRs:/ {printf "%s %s\n", name, $0}'
