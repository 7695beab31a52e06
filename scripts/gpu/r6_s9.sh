set -o pipefail
mkdir -p gpurun_out/r6s9
for m in 0 0b 1; do
  g=${m%b}
  DET_HIP_GRAPH=$g timeout -k 10 300 python -u scripts/dbg/graph_vs_eager_resnet.py --out gpurun_out/r6s9/t$m.pt --steps 12 --bs 128 --image 224 > gpurun_out/r6s9/t$m.log 2>&1 || { echo "run $m failed rc=$?"; tail -20 gpurun_out/r6s9/t$m.log; exit 1; }
  if grep -q "Segmentation\|Fatal Python" gpurun_out/r6s9/t$m.log; then echo crash; exit 1; fi
done
python scripts/dbg/graph_vs_eager_resnet.py --compare gpurun_out/r6s9/t0.pt gpurun_out/r6s9/t0b.pt > gpurun_out/r6s9/cmp_eager.txt
python scripts/dbg/graph_vs_eager_resnet.py --compare gpurun_out/r6s9/t0.pt gpurun_out/r6s9/t1.pt > gpurun_out/r6s9/cmp_graph.txt
cat gpurun_out/r6s9/cmp_eager.txt gpurun_out/r6s9/cmp_graph.txt
