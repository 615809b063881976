# abtree/<A> (an older tree with its built library) against this tree on the 4K, C3 and C2 lines,
# alternating.  bash tools/r5/tree_ab.sh <outdir> <A> <reps> <lines: any of 4k,c3,c2>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5tree}; A=${2:-r5p}; R=${3:-1}; L=${4:-4k,c3}; mkdir -p $O
for rep in $(seq 1 $R); do
  for v in a b; do
    if [ $v = a ]; then D=abtree/$A; else D=.; fi
    case ",$L," in *,4k,*) (cd $D && timeout -k 10 150 python bench.py --steps 100 --warmup 10 --width 3840 --height 2160 --batch 1 --ring 2 --no-secondary --no-cpu-baseline) > $O/4k_${v}_$rep.json 2> $O/4k_${v}_$rep.err || exit 1;; esac
    case ",$L," in *,c3,*) (cd $D && timeout -k 10 200 python tools/bench_c3.py --steps 10 --json $O/c3_${v}_$rep.json) > /dev/null 2> $O/c3_${v}_$rep.err || exit 1;; esac
    case ",$L," in *,c2,*) (cd $D && timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline) > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 1;; esac
  done
done
