#!/bin/bash
# Round 6 closing set: C2 and world-1 fused A/B against abtree/prev (one box, alternating), then
# the measurement set of tools/r6/final_c.sh on this build.
#   bash tools/r6/final_d.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=${1:-r6final4}
TESTS=none LINES=c2 bash tools/r6/lib_ab.sh $O/ab 2 prev . || exit 1
for v in prev .; do
  t=$([ $v = . ] && echo cur || echo $v); d=$([ $v = . ] && echo . || echo abtree/$v)
  (cd $d && RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29570 + RANDOM % 100)) \
      timeout -k 10 200 python bench.py --gpus 1 --dist --steps 1000 --warmup 50 --no-secondary \
      --no-cpu-baseline --no-kernel-timing) > gpurun_out/$O/ab/dist_$t.json 2> gpurun_out/$O/ab/dist_$t.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/$O/ab/dist_$t.json').read().strip().splitlines()[-1]);print('dist_$t', d['value'])"
done
bash tools/r6/final_c.sh $O
