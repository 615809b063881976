# A/B timing of two builds of libgdf.so (lib_a, lib_b) on one box, alternating, long runs.
# usage: bash tools/ab_bench.sh OUTDIR [bench args...]
O=$1; shift; mkdir -p $O
L=ros_gpu_depthmap_fusion_amd/lib
cp $L/libgdf.so $O/.keep.so
for r in 1 2 3; do
  for v in a b; do
    cp ros_gpu_depthmap_fusion_amd/lib_$v/libgdf.so $L/libgdf.so
    timeout -k 10 120 python bench.py --gpus 1 --no-secondary --no-cpu-baseline --no-kernel-timing "$@" > $O/$v$r.json 2>/dev/null || exit 1
  done
done
cp $O/.keep.so $L/libgdf.so
