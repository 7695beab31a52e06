set -o pipefail
O=gpurun_out/r6s19; mkdir -p $O
timeout -k 10 120 python -u scripts/dbg/memset_graph_repro.py > $O/memset.txt 2>&1 || { echo memset failed; tail $O/memset.txt; exit 1; }
grep -v amdgpu.ids $O/memset.txt
timeout -k 10 200 python -u scripts/dbg/miopen_graph_repro.py --step > $O/miopen_step.txt 2>&1 || { echo miopen failed; tail $O/miopen_step.txt; exit 1; }
timeout -k 10 200 python -u scripts/dbg/miopen_graph_repro.py --step --fix-memsets > $O/miopen_step_fixed.txt 2>&1 || { echo miopen fixed failed; tail $O/miopen_step_fixed.txt; exit 1; }
echo "--- miopen step"; grep -v amdgpu.ids $O/miopen_step.txt | tail -5; echo "--- fixed"; grep -v amdgpu.ids $O/miopen_step_fixed.txt | tail -6
run() {
  local name=$1 g=$2; shift 2
  DET_HIP_GRAPH=$g timeout -k 10 300 python -u scripts/dbg/graph_vs_eager_resnet.py --out $O/$name.pt "$@" > $O/$name.log 2>&1 || { echo "run $name failed"; tail -20 $O/$name.log; return 1; }
  if grep -q "Segmentation\|Fatal Python" $O/$name.log; then echo crash; return 1; fi
}
run e 0 --steps 30 --bs 512 && run g 1 --steps 30 --bs 512 &&
python scripts/dbg/graph_vs_eager_resnet.py --compare $O/e.pt $O/g.pt > $O/cmp.txt && tail -6 $O/cmp.txt
