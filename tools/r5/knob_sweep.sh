# Round-5 default check: the C2 line (300 / 30) under single-knob variants, 2 reps alternating.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/env_sweep.sh gpurun_out/${1:-r5knobs} "GDF_X=0" "GDF_RUN_HIST_SORT=1" "GDF_RUN_HIST_ALL=1" "GDF_GROUP_FIRST=1" "GDF_RUN_WAVE=1" "GDF_RUN_Q16=1" "GDF_GROUP_BLOCKS=1024" "GDF_SORT_BLOCKS=1024" "GDF_GRID_WPT=4" "GDF_SMALL_GROUP=64" "GDF_RUN_STAGE=512" "GDF_RUN_BIG_BLOCKS=512" -- --steps 300 --warmup 30
