set -o pipefail
mkdir -p gpurun_out/r6s10
run() {  # name graph args...
  local name=$1 g=$2; shift 2
  DET_HIP_GRAPH=$g timeout -k 10 300 python -u scripts/dbg/graph_vs_eager_resnet.py --out gpurun_out/r6s10/$name.pt "$@" > gpurun_out/r6s10/$name.log 2>&1 || { echo "run $name failed"; tail -20 gpurun_out/r6s10/$name.log; return 1; }
  if grep -q "Segmentation\|Fatal Python" gpurun_out/r6s10/$name.log; then echo crash; return 1; fi
}
run e_step 0 --steps 30 --bs 512 && run g_step 1 --steps 30 --bs 512 &&
python scripts/dbg/graph_vs_eager_resnet.py --compare gpurun_out/r6s10/e_step.pt gpurun_out/r6s10/g_step.pt > gpurun_out/r6s10/cmp_step.txt &&
run e_one 0 --steps 30 --bs 512 --one-workload 5 && run g_one 1 --steps 30 --bs 512 --one-workload 5 &&
python scripts/dbg/graph_vs_eager_resnet.py --compare gpurun_out/r6s10/e_one.pt gpurun_out/r6s10/g_one.pt > gpurun_out/r6s10/cmp_one.txt &&
tail -4 gpurun_out/r6s10/cmp_step.txt && cat gpurun_out/r6s10/cmp_one.txt
