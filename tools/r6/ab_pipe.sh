#!/bin/bash
# Round 6: lib_ab.sh (C2 only) and then C2 at 2 and 4 batches in flight on this tree.
#   bash tools/r6/ab_pipe.sh OUT REPS VARIANT...
set -o pipefail
O=$1; shift
LINES=c2 bash tools/r6/lib_ab.sh $O "$@" || exit 1
for p in 2 4; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --no-secondary --no-cpu-baseline \
      --no-kernel-timing --pipeline $p > gpurun_out/$O/c2_pipe$p.json 2> gpurun_out/$O/c2_pipe$p.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/$O/c2_pipe$p.json').read().strip().splitlines()[-1]);print('pipe$p', d['value'])"
done
