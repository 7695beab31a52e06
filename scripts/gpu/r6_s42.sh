#!/bin/bash
# Round-6 session 42: Linear bias gradients from the hipBLASLt BGRADB epilogue: transformer GPU tests,
# then BERT bench A/B (DET_BGRAD_EPILOGUE 1 / 0) under hipGraph, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s42; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_trial_resume.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1; rc=$?
tail -2 $O/test.log; grep -E "FAILED|Error" $O/test.log | head -10
[ $rc -eq 0 ] || exit $rc
python -c "
import torch
from determined_1_amd.ops import transformer as t
x=torch.randn(4608,768,device='cuda',dtype=torch.bfloat16,requires_grad=True); w=torch.randn(2304,768,device='cuda',dtype=torch.bfloat16,requires_grad=True); b=torch.zeros(2304,device='cuda',dtype=torch.bfloat16,requires_grad=True)
t.NATIVE_LINEAR=False
t.linear(x,w,b).sum().backward(); print('bgrad counts', t.LINEAR_BGRAD_COUNTS)"
for i in 1 2; do
  for v in 1 0; do
    DET_BGRAD_EPILOGUE=$v timeout -k 10 300 python -u scripts/bench_bert.py --steps 100 --warmup 10 --hip-graph > $O/bert_$v.$i.json 2> $O/bert.err || { tail $O/bert.err; exit 1; }
    echo "bgrad_epilogue=$v: $(tail -1 $O/bert_$v.$i.json | python -c 'import sys,json; print(json.loads(sys.stdin.read())["value"])')"
  done
done
