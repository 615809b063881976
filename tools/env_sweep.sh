# Long-run bench under several environment settings of one build (tuning knobs), repeated.
# usage: bash tools/env_sweep.sh OUTDIR "VAR=val ..." "VAR=val ..." -- [bench args...]
O=$1; shift; mkdir -p $O
V=(); while [ "$1" != "--" ]; do V+=("$1"); shift; done; shift
for r in 1 2; do
  i=0
  for v in "${V[@]}"; do
    env $v timeout -k 10 120 python bench.py --gpus 1 --no-secondary --no-cpu-baseline --no-kernel-timing "$@" > $O/v${i}_$r.json 2>/dev/null || exit 1
    i=$((i+1))
  done
done
