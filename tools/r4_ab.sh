# A/B of a build on the C2 line: GPU parity subset, then the 300-step line twice (per-kernel
# event timing on), the mask kernel's average from the line's roofline.per_kernel.
#   bash tools/r4_ab.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r4ab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_round4.py > $O/t.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline > $O/c2.$rep.json 2> $O/c2.$rep.err || exit 1
done
tail -n 1 $O/t.log
