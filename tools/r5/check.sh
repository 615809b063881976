# GPU suite, then A/B of this tree against abtree/<A> (C2 300 steps, alternating), then the C2
# kernel trace with one batch in flight.  bash tools/r5/check.sh <outdir> [A]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5chk}; A=${2:-r4}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/pytest_gpu.log 2>&1 || exit 1
for i in 1 2; do
  (cd abtree/$A && timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline) > $O/a$i.json 2> $O/a$i.err || exit 1
  timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline > $O/b$i.json 2> $O/b$i.err || exit 1
done
B="bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/p1 -o run --output-format csv -- python3 $B > $O/p1.json 2> $O/p1.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t4k -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --width 3840 --height 2160 --batch 1 --ring 2 --pipeline 1 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/t4k.json 2> $O/t4k.err || exit 1
