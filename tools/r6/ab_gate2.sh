#!/bin/bash
# Round 6: grid gate variants A/B on one box (2000 steps each, alternating):
# spin = the tickets alone, gate = wait for the previous update's end, early = wait until the
# previous update is next in its stream.
set -o pipefail
O=gpurun_out/${1:-r6e}; mkdir -p $O
timeout -k 10 300 env GDF_GRID_GATE_EARLY=1 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_round4.py -k "batch8" > $O/pytest_early.log 2>&1 || { tail -30 $O/pytest_early.log; exit 1; }
tail -2 $O/pytest_early.log
for r in 1 2 3; do
  for v in spin early gate; do
    unset GDF_GRID_SPIN GDF_GRID_GATE_EARLY
    [ $v = spin ] && export GDF_GRID_SPIN=1
    [ $v = early ] && export GDF_GRID_GATE_EARLY=1
    timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --no-secondary --no-cpu-baseline \
        --no-kernel-timing > $O/$v$r.json 2> $O/$v$r.err || exit 1
    python -c "import json;d=json.loads(open('$O/$v$r.json').read().strip().splitlines()[-1]);print('$v$r',d['value'])"
  done
done
