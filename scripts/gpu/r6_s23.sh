set -o pipefail
O=gpurun_out/r6s23; mkdir -p $O
for bs in 512 768 1024; do
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --batch-per-gpu $bs > $O/bs$bs.json 2> $O/bs$bs.err || { echo "bs $bs failed"; tail -5 $O/bs$bs.err; exit 1; }
  tail -1 $O/bs$bs.json | cut -c1-330
done
