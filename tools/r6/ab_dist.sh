#!/bin/bash
# Round 6: the parity tests of the fused step, then A/B of the world-1 fused line (--dist, RCCL
# from libgdf) on one box, alternating, plus C2 for each variant.
#   bash tools/r6/ab_dist.sh OUT REPS VARIANT...   (VARIANT: abtree/<name> or .)
set -o pipefail
O=$PWD/gpurun_out/$1; R=$2; shift 2; V="$@"
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_local_world.py "tests/test_gpu_round4.py::test_partition_runs_voxelize_runs_match_oracle" \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
dir() { if [ $1 = . ]; then echo .; else echo abtree/$1; fi; }
tag() { if [ $1 = . ]; then echo cur; else echo $1; fi; }
port=29561
for rep in $(seq 1 $R); do
  for v in $V; do
    t=$(tag $v); port=$((port + 1))
    (cd $(dir $v) && RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 \
        MASTER_PORT=$port timeout -k 10 200 python bench.py --gpus 1 --dist --steps 1000 --warmup 50 \
        --no-secondary --no-cpu-baseline --no-kernel-timing) > $O/dist_$t$rep.json 2> $O/dist_$t$rep.err || exit 1
    python -c "import json;d=json.loads(open('$O/dist_$t$rep.json').read().strip().splitlines()[-1]);print('dist_$t$rep', d['value'])"
  done
done
