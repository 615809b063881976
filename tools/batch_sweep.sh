O=gpurun_out/bsw; mkdir -p $O
for b in 6 8 12; do
  timeout -k 10 120 python bench.py --gpus 1 --no-secondary --no-cpu-baseline --no-kernel-timing --steps 1500 --warmup 50 --batch $b > $O/b$b.json 2>/dev/null || exit 1
done
