# Wave mode of k_group_runs_big (default) against GDF_RUN_WAVE_MODE=0 (block mode for every queued
# group) on one box: the long-group tests, group traces of C3 / 4K, then the 4K single-frame line,
# the C3 line and the C2 line, alternating.  bash tools/r5/wave_ab.sh <outdir> [reps]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5wave}; R=${2:-2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_round3.py tests/test_gpu_round4.py -k "c3 or adversarial or 4k or batch8" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/group_trace.py --c3 256 > $O/gt_c3.txt 2>&1 || exit 1
timeout -k 10 200 python tools/group_trace.py 3840 2160 4 > $O/gt_4k.txt 2>&1 || exit 1
for rep in $(seq 1 $R); do
  for v in wave block; do
    if [ $v = block ]; then E="GDF_RUN_WAVE_MODE=0"; else E="GDF_X=0"; fi
    env $E timeout -k 10 150 python bench.py --steps 100 --warmup 10 --width 3840 --height 2160 --batch 1 --ring 2 --no-secondary --no-cpu-baseline > $O/4k_${v}_$rep.json 2> $O/4k_${v}_$rep.err || exit 1
    env $E timeout -k 10 200 python tools/bench_c3.py --steps 10 --json $O/c3_${v}_$rep.json > /dev/null 2> $O/c3_${v}_$rep.err || exit 1
    env $E timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 1
  done
done
