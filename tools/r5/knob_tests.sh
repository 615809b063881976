# The knob parity tests on this tree's library.  bash tools/r5/knob_tests.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5knobtests}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "knobs or frame_sort or adversarial" > $O/pytest_knobs.log 2>&1
