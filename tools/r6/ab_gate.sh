#!/bin/bash
# Round 6: the grid-update stream gate - parity subset, then A/B against the ticket spin
# (GDF_GRID_SPIN=1) on one box, alternating, 2000 steps each; then pipeline 4.
set -o pipefail
O=gpurun_out/${1:-r6d}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_round4.py tests/test_gpu_local_world.py tests/test_gpu_parity.py tests/test_gpu_round5.py \
    > $O/pytest_subset.log 2>&1 || { tail -30 $O/pytest_subset.log; exit 1; }
tail -3 $O/pytest_subset.log
for r in 1 2 3; do
  for v in gate spin; do
    if [ $v = spin ]; then export GDF_GRID_SPIN=1; else unset GDF_GRID_SPIN; fi
    timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --no-secondary --no-cpu-baseline \
        --no-kernel-timing > $O/$v$r.json 2> $O/$v$r.err || exit 1
    python -c "import json;d=json.loads(open('$O/$v$r.json').read().strip().splitlines()[-1]);print('$v$r',d['value'])"
  done
done
unset GDF_GRID_SPIN
for v in gate spin; do
  if [ $v = spin ]; then export GDF_GRID_SPIN=1; else unset GDF_GRID_SPIN; fi
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --pipeline 4 --no-secondary --no-cpu-baseline \
      --no-kernel-timing > $O/p4_$v.json 2> $O/p4_$v.err || exit 1
  python -c "import json;d=json.loads(open('$O/p4_$v.json').read().strip().splitlines()[-1]);print('p4_$v',d['value'])"
done
