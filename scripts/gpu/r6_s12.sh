set -o pipefail
mkdir -p gpurun_out/r6s12
run() {  # name graph args...
  local name=$1 g=$2; shift 2
  DET_HIP_GRAPH=$g timeout -k 10 300 python -u scripts/dbg/graph_vs_eager_resnet.py --out gpurun_out/r6s12/$name.pt "$@" > gpurun_out/r6s12/$name.log 2>&1 || { echo "run $name failed"; tail -20 gpurun_out/r6s12/$name.log; return 1; }
  if grep -q "Segmentation\|Fatal Python" gpurun_out/r6s12/$name.log; then echo crash; return 1; fi
}
run e 0 --steps 8 --bs 512 && run g 1 --steps 8 --bs 512 && DET_GRAPH_SINK=0 run gns 1 --steps 8 --bs 512 &&
python scripts/dbg/graph_vs_eager_resnet.py --compare gpurun_out/r6s12/e.pt gpurun_out/r6s12/gns.pt > gpurun_out/r6s12/cmp_nosink.txt &&
cat gpurun_out/r6s12/cmp_nosink.txt
