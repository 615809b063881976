# The k_mask knobs again after the camera lookup: the C2 line (300 / 30), 2 reps alternating.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/env_sweep.sh gpurun_out/${1:-r5knobs2} "GDF_X=0" "GDF_MASK_OCC8=0" "GDF_MASK_ROWS=2" "GDF_RUN_HIST_ALL=1" "GDF_GROUP_FIRST=1" -- --steps 300 --warmup 30
