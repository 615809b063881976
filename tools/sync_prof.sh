# component-sync timelines: kernel + copy traces of tools/sync_probe.py, default and GDF_DL_FORK=1
set -o pipefail
O=gpurun_out/${1:-syncprof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 python tools/sync_probe.py 400 > $O/base.txt 2>&1 || exit 1
GDF_DL_FORK=1 timeout -k 10 60 python tools/sync_probe.py 400 > $O/fork.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/base -o run -- python3 tools/sync_probe.py 200 > $O/base_prof.txt 2>&1 || exit 1
