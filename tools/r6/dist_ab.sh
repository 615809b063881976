#!/bin/bash
# Round 6: the fused step's receive side folded into the rebase pass - the multi-rank tests, then
# the world-1 --dist line, abtree/<A> (before) against this tree, alternating.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r6h}; A=${2:-r6base}; R=${3:-3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_local_world.py tests/test_gpu_multi.py > $O/pytest_multi.log 2>&1 || { tail -30 $O/pytest_multi.log; exit 1; }
tail -2 $O/pytest_multi.log
E="RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1"
for rep in $(seq 1 $R); do
  for v in a b; do
    if [ $v = a ]; then D=abtree/$A; else D=.; fi
    (cd $D && env $E MASTER_PORT=$((29530 + rep)) timeout -k 10 240 python bench.py --gpus 1 --dist --steps 1000 --warmup 50 --no-secondary --no-cpu-baseline --no-kernel-timing) > $O/${v}_n1_$rep.json 2> $O/${v}_n1_$rep.err || exit 1
    python -c "import json;d=json.loads(open('$O/${v}_n1_$rep.json').read().strip().splitlines()[-1]);print('$v',$rep,d['value'])"
  done
done
(env $E GDF_SORT_PT=8 MASTER_PORT=29541 timeout -k 10 240 python bench.py --gpus 1 --dist --steps 1000 --warmup 50 --no-secondary --no-cpu-baseline --no-kernel-timing) > $O/b_n1_pt8.json 2> $O/b_n1_pt8.err
timeout -k 10 240 python bench.py --gpus 4 --transport local --steps 100 --warmup 10 --no-secondary --no-cpu-baseline > $O/local4.json 2> $O/local4.err || exit 1
python -c "import json;d=json.loads(open('$O/local4.json').read().strip().splitlines()[-1]);print('local4',d['value'])"
python -c "import json;d=json.loads(open('$O/b_n1_pt8.json').read().strip().splitlines()[-1]);print('pt8',d['value'])"
