#!/bin/bash
# measurement-only builds of layer_ops.hip with QZ_ATTN_ABL=<n> (scripts/dev/attn_ablation.py)
set -e
cd "$(dirname "$0")/../../quantizations_amd/csrc"
for a in 0 1 2 4 8 16 32; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-rdc -shared \
    -DQZ_ATTN_ABL=$a -o ../../scripts/dev/attn_abl/libattn_$a.so layer_ops.hip &
done
wait
