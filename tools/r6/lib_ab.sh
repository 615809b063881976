#!/bin/bash
# Round 6: A/B(/C...) of builds on one box, alternating.  Each variant is a tree: abtree/<name> (a
# git archive of an earlier state with its built library) or "." (this tree).  First the parity
# subset on this tree (TESTS=none skips it), then per rep C2 (2000 steps) for every variant, then
# once per variant C2 with kernel timing, 4K single frames and the C3 line (LINES=c2 skips those).
#   usage: TESTS="..." LINES=all bash tools/r6/lib_ab.sh OUT REPS VARIANT...
set -o pipefail
O=$PWD/gpurun_out/$1; R=$2; shift 2; V="$@"
T=${TESTS:-tests/test_gpu_round4.py tests/test_gpu_round3.py tests/test_gpu_parity.py tests/test_gpu_round5.py}
mkdir -p $O
if [ "$T" != none ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread $T \
      > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
show() { python -c "
import json,sys;d=json.loads(open('$1').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('$2', d['value'], round(d['ms_per_step']*1e3,2), r.get('per_kernel_us') or {k:(v.get('us'),v.get('GBps')) for k,v in (r.get('per_kernel') or {}).items()})"; }
dir() { if [ $1 = . ]; then echo .; else echo abtree/$1; fi; }
tag() { if [ $1 = . ]; then echo cur; else echo $1; fi; }
for rep in $(seq 1 $R); do
  for v in $V; do
    t=$(tag $v)
    (cd $(dir $v) && timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --no-secondary \
        --no-cpu-baseline --no-kernel-timing) > $O/c2_$t$rep.json 2> $O/c2_$t$rep.err || exit 1
    show $O/c2_$t$rep.json c2_$t$rep
  done
done
[ "${LINES:-all}" = c2 ] && exit 0
for v in $V; do
  t=$(tag $v)
  (cd $(dir $v) && timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-secondary \
      --no-cpu-baseline) > $O/c2k_$t.json 2> $O/c2k_$t.err || exit 1
  show $O/c2k_$t.json c2k_$t
  (cd $(dir $v) && timeout -k 10 200 python bench.py --width 3840 --height 2160 --batch 1 --steps 200 \
      --warmup 20 --no-secondary --no-cpu-baseline) > $O/4k_$t.json 2> $O/4k_$t.err || exit 1
  show $O/4k_$t.json 4k_$t
  (cd $(dir $v) && timeout -k 10 300 python tools/bench_c3.py --steps 20) > $O/c3_$t.json 2> $O/c3_$t.err || exit 1
  show $O/c3_$t.json c3_$t
done
