set -o pipefail
mkdir -p gpurun_out/r6s13
DET_HIP_GRAPH=1 timeout -k 10 300 python -u scripts/dbg/graph_vs_eager_resnet.py --out gpurun_out/r6s13/g.pt --steps 6 --bs 512 --trace-sink > gpurun_out/r6s13/g.log 2>&1 && grep -v amdgpu.ids gpurun_out/r6s13/g.log | tail -40 &&
DET_HIP_GRAPH=1 timeout -k 10 300 python -u scripts/dbg/graph_vs_eager_resnet.py --out gpurun_out/r6s13/g128.pt --steps 6 --bs 128 --trace-sink > gpurun_out/r6s13/g128.log 2>&1 && grep -v amdgpu.ids gpurun_out/r6s13/g128.log | tail -40
