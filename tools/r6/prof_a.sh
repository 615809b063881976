#!/bin/bash
# Round 6 measurement record: the gate knob tests, SQ counters of the C2 step (refreshing
# profiles/pmc_sq.json after the camera lookup) and of the C3 window's k_sel, the 4K group trace
# (longest voxel, chain floor).   bash tools/r6/prof_a.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r6f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_round4.py -k "GRID_GATE or grid_mirror or tuning" > $O/pytest_gate.log 2>&1 || { tail -30 $O/pytest_gate.log; exit 1; }
tail -2 $O/pytest_gate.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/sq_c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1 > $O/sq_c2.json 2> $O/sq_c2.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc $SQ -d $O/sq_c3 -o run --output-format csv -- python3 tools/bench_c3.py --steps 3 --profile-steps 1 > $O/sq_c3.out 2> $O/sq_c3.err || exit 1
timeout -k 10 180 python tools/group_trace.py 3840 2160 4 dense > $O/gtrace_4k.txt 2>&1 || exit 1
head -8 $O/gtrace_4k.txt
find $O -name "*counter_collection.csv" | head
