set -o pipefail
mkdir -p gpurun_out/r6s15
run() {  # name graph args...
  local name=$1 g=$2; shift 2
  DET_HIP_GRAPH=$g timeout -k 10 300 python -u scripts/dbg/graph_vs_eager_resnet.py --out gpurun_out/r6s15/$name.pt "$@" > gpurun_out/r6s15/$name.log 2>&1 || { echo "run $name failed"; tail -20 gpurun_out/r6s15/$name.log; return 1; }
  if grep -q "Segmentation\|Fatal Python" gpurun_out/r6s15/$name.log; then echo crash; return 1; fi
}
fcb() { python - "$@" <<'PY'
import sys, torch
a = torch.load(sys.argv[1], weights_only=True); b = torch.load(sys.argv[2], weights_only=True)
r = []
for s in range(len(a["fcb"])):
    (ga, pa), (gb, pb) = a["fcb"][s][0], b["fcb"][s][0]
    r.append(round(float((ga - gb).abs().max() / ga.abs().max()), 4))
print(sys.argv[2], "fc.bias grad rel per step", r, "graph", b.get("graph"))
PY
}
run e 0 --steps 7 --bs 512 &&
DET_SINK_CAPTURE_FOREACH=0 run g_loop 1 --steps 7 --bs 512 && fcb gpurun_out/r6s15/e.pt gpurun_out/r6s15/g_loop.pt &&
DET_GRAPH_KEEP=1 run g_keep 1 --steps 7 --bs 512 --dump-nodes && fcb gpurun_out/r6s15/e.pt gpurun_out/r6s15/g_keep.pt && grep -A40 "graph nodes" gpurun_out/r6s15/g_keep.log | head -60
