#!/bin/bash
# Round 6: k_sel keeping its run-detection keys in LDS - the rollbuffer parity tests, then the C3
# line with and without (GDF_NO_SEL_KEY_LDS), alternating on one box.
set -o pipefail
O=gpurun_out/${1:-r6i}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_round3.py tests/test_gpu_parity.py tests/test_facade_gpu.py > $O/pytest_sel.log 2>&1 || { tail -30 $O/pytest_sel.log; exit 1; }
tail -2 $O/pytest_sel.log
for r in 1 2; do
  for v in lds recompute; do
    unset GDF_NO_SEL_KEY_LDS
    [ $v = recompute ] && export GDF_NO_SEL_KEY_LDS=1
    timeout -k 10 300 python tools/bench_c3.py --steps 20 > $O/c3_$v$r.json 2> $O/c3_$v$r.err || exit 1
    python -c "
import json;d=json.loads(open('$O/c3_$v$r.json').read().strip().splitlines()[-1])
pk=d.get('roofline',{}).get('per_kernel',{})
print('$v$r', d['value'], d['ms_per_step'], {k:(v.get('us'),v.get('GBps')) for k,v in pk.items() if k in ('sel','group','sort')})"
  done
done
