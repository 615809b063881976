# GPU suite, then packed run keys (default) against GDF_NO_PACK_RUNS on one box: C2 300-step lines,
# the 4K single-frame line and the C3 line, alternating.  bash tools/r5/pack_ab.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5pack}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for rep in 1 2; do
  for v in pack nopack; do
    if [ $v = nopack ]; then E="GDF_NO_PACK_RUNS=1"; else E="GDF_X=0"; fi
    env $E timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 1
    env $E timeout -k 10 150 python bench.py --steps 100 --warmup 10 --width 3840 --height 2160 --batch 1 --ring 2 --no-secondary --no-cpu-baseline > $O/4k_${v}_$rep.json 2> $O/4k_${v}_$rep.err || exit 1
    env $E timeout -k 10 200 python tools/bench_c3.py --steps 10 --json $O/c3_${v}_$rep.json > /dev/null 2> $O/c3_${v}_$rep.err || exit 1
  done
done
