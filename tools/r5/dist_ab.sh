# The fused C++ step, abtree/<A> against this tree, alternating: the world-1 RCCL --dist line and
# the in-process 4-rank line (--transport local).  bash tools/r5/dist_ab.sh <outdir> <A> [reps]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5distab}; A=${2:-r5p}; R=${3:-2}; mkdir -p $O
E="RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1"
for rep in $(seq 1 $R); do
  for v in a b; do
    if [ $v = a ]; then D=abtree/$A; else D=.; fi
    (cd $D && env $E MASTER_PORT=$((29530 + rep)) timeout -k 10 240 python bench.py --gpus 1 --dist --steps 300 --warmup 30 --no-secondary --no-cpu-baseline) > $O/${v}_n1_$rep.json 2> $O/${v}_n1_$rep.err || exit 1
    (cd $D && timeout -k 10 240 python bench.py --gpus 4 --transport local --steps 100 --warmup 10 --no-secondary --no-cpu-baseline) > $O/${v}_local4_$rep.json 2> $O/${v}_local4_$rep.err || exit 1
  done
done
