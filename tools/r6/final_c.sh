#!/bin/bash
# Round-6 final measurement set on the last build: GPU suite + smoke, the default line (python
# bench.py: 300 / 30, every secondary, CPU baseline), the driver's short line (20 / 5), the world-1
# --dist line, the kernel trace of the C2 step with one batch in flight (the line's roofline
# kernel), PMC FETCH / WRITE of it, the 4K trace, the C3 line + its k_sel phase trace.
#   bash tools/r6/final_c.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r6final2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 timeout -k 10 240 python bench.py --gpus 1 --dist --steps 300 --warmup 30 --no-secondary --no-cpu-baseline > $O/dist_n1.json 2> $O/dist_n1.err || exit 1
B="bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O/trace.json 2> $O/trace.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B > $O/fetch.json 2> $O/fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B > $O/write.json 2> $O/write.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t4k -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --width 3840 --height 2160 --batch 1 --ring 2 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/t4k.json 2> $O/t4k.err || exit 1
timeout -k 10 200 python tools/bench_c3.py --steps 10 --json $O/c3.json > /dev/null 2>> $O/c3.err || exit 1
timeout -k 10 300 python tools/sel_trace.py 256 > $O/seltrace.txt 2>&1 || exit 1
for f in bench_default bench_20_5 dist_n1; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"; done
