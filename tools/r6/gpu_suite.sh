#!/bin/bash
# Round 6: the whole GPU suite, then the C2 line (300 steps, no secondary lines).
set -o pipefail
out=gpurun_out/${1:-r6c}
mkdir -p $out
timeout -k 10 1500 python -u -m pytest -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread \
    tests > $out/pytest_gpu.log 2>&1
rc=$?
tail -25 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline \
    > $out/bench_300.json 2> $out/bench_300.err
rc=$?
cat $out/bench_300.json | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
exit $rc
