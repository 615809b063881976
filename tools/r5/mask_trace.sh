# k_mask_px phase stamps (diagnostic library) on one isolated C2 batch and one 4K frame.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5masktrace}; mkdir -p $O
timeout -k 10 120 python tools/mask_trace.py 640 480 8 dense > $O/c2.txt 2>&1 || exit 1
timeout -k 10 120 python tools/mask_trace.py 3840 2160 1 dense > $O/4k.txt 2>&1 || exit 1
