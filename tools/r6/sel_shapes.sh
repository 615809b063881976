#!/bin/bash
# Round 6: k_sel tile shapes on the C3 line (GDF_SEL_SHAPE "segs,threads"), current build.
set -o pipefail
O=gpurun_out/${1:-r6j}; shift; mkdir -p $O
for sh in default 16,512 8,1024 8,512 16,256 4,1024 default; do
  tag=${sh/,/x}
  if [ "$sh" = default ]; then unset GDF_SEL_SHAPE; else export GDF_SEL_SHAPE=$sh; fi
  timeout -k 10 240 python tools/bench_c3.py --steps 15 > $O/c3_$tag.json 2>> $O/c3_$tag.err || exit 1
  python -c "
import json;d=json.loads(open('$O/c3_$tag.json').read().strip().splitlines()[-1])
pk=d['roofline']['per_kernel']; print('$sh', d['value'], d['ms_per_step'], 'sel', pk['sel']['avg_us'], pk['sel']['GBps'])"
done
