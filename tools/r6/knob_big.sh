#!/bin/bash
# Round 6: the long-group kernel's grid on C2 (a VGA batch queues no group: the launch is a link of
# the chain with nothing to do) and the group-phase grid - 2000-step C2 lines, alternating.
set -o pipefail
O=gpurun_out/${1:-knobbig}; mkdir -p $O
V=("GDF_X=0" "GDF_GROUP_SCAN_TILES=1000000" "GDF_GROUP_SCAN_TILES=1000000 GDF_GROUP_BLOCKS=512" "GDF_GROUP_SCAN_TILES=1000000 GDF_RUN_BIG_BLOCKS=32")
for r in 1 2; do
  i=0
  for v in "${V[@]}"; do
    env $v timeout -k 10 150 python bench.py --gpus 1 --steps 2000 --warmup 100 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/v${i}_$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('$O/v${i}_$r.json').read().strip().splitlines()[-1]);print('$v', $r, d['value'])"
    i=$((i+1))
  done
done
