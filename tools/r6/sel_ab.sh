#!/bin/bash
# Round 6: k_sel A/B - the rollbuffer parity tests,
# the per-tile phase trace of the C3 window, then the C3 line of abtree/<A> (before) and this tree.
#   usage: bash tools/r6/sel_lag.sh OUT [A]
set -o pipefail
O=$PWD/gpurun_out/$1; A=${2:-base}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_round3.py tests/test_gpu_parity.py tests/test_facade_gpu.py tests/test_gpu_round5.py \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_local_world.py -k "sharded or rollbuffer" > $O/pytest_lw.log 2>&1 || { tail -30 $O/pytest_lw.log; exit 1; }
tail -1 $O/pytest_lw.log
timeout -k 10 300 python tools/sel_trace.py 256 > $O/seltrace.txt 2>&1 || { tail -20 $O/seltrace.txt; exit 1; }
cat $O/seltrace.txt
for r in 1 2; do
  for v in $A .; do
    t=$([ $v = . ] && echo cur || echo $v); d=$([ $v = . ] && echo . || echo abtree/$v)
    (cd $d && timeout -k 10 300 python tools/bench_c3.py --steps 20) > $O/c3_$t$r.json 2> $O/c3_$t$r.err || exit 1
    python -c "import json;d=json.loads(open('$O/c3_$t$r.json').read().strip().splitlines()[-1]);print('$t$r', d['value'], d['ms_per_step'], d['roofline']['per_kernel']['sel'])"
  done
done
