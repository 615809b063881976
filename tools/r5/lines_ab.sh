# Env variants ("base" = none) on the 4K single-frame line, the C3 line and the C2 line, alternating
# on one box.  bash tools/r5/lines_ab.sh <outdir> <reps> <lines: any of 4k,c3,c2> v1 v2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5lines}; R=${2:-1}; L=${3:-4k,c3,c2}; shift 3; mkdir -p $O
for rep in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    i=$((i+1)); echo "v$i: $v" > $O/v$i.name
    if [ "$v" = base ]; then E="GDF_X=0"; else E="$v"; fi
    case ",$L," in *,4k,*) env $E timeout -k 10 150 python bench.py --steps 100 --warmup 10 --width 3840 --height 2160 --batch 1 --ring 2 --no-secondary --no-cpu-baseline > $O/4k_v${i}_$rep.json 2> $O/4k_v${i}_$rep.err || exit 1;; esac
    case ",$L," in *,c3,*) env $E timeout -k 10 200 python tools/bench_c3.py --steps 10 --json $O/c3_v${i}_$rep.json > /dev/null 2> $O/c3_v${i}_$rep.err || exit 1;; esac
    case ",$L," in *,c2,*) env $E timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline > $O/c2_v${i}_$rep.json 2> $O/c2_v${i}_$rep.err || exit 1;; esac
  done
done
