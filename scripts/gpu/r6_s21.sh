set -o pipefail
O=gpurun_out/r6s21; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 > $O/graph_$i.json 2> $O/graph_$i.err || { echo graph bench failed; tail $O/graph_$i.err; exit 1; }
  tail -1 $O/graph_$i.json
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-hip-graph > $O/eager_$i.json 2> $O/eager_$i.err || { echo eager bench failed; tail $O/eager_$i.err; exit 1; }
  tail -1 $O/eager_$i.json
done
