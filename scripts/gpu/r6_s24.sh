#!/bin/bash
# Round-6 session 24: detection trials with the backbone/FPN/head convolutions on the native conv
# kernels (DET_NATIVE_CONV2D=1, default) vs MIOpen (=0), bf16 O2 and fp32 O0, same box back to back.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s24; mkdir -p $O
export TMPDIR=/tmp
for m in maskrcnn retinanet detr fasterrcnn; do
  for amp in O2 O0; do
    for nc in 1 0; do
      DET_NATIVE_CONV2D=$nc timeout -k 10 400 python -u scripts/bench_detection.py --model $m --amp $amp --steps 30 --warmup 10 > $O/${m}_${amp}_nc$nc.json 2> $O/${m}_${amp}_nc$nc.err || { echo "$m $amp nc=$nc failed"; tail -8 $O/${m}_${amp}_nc$nc.err; exit 1; }
      echo "$m $amp native=$nc: $(tail -1 $O/${m}_${amp}_nc$nc.json | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["config"].get("s_per_iter"), d["config"].get("native_conv2d"))')"
    done
  done
done
