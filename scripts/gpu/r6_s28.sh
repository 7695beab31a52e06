#!/bin/bash
# Round-6 session 28: igemm8 (eight-phase schedule on the implicit-GEMM gather, cfg 21): numerics on
# every cfg test shape, then the ResNet-50 3x3 pass timings with the default configs vs cfg 21 forced.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s28; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_igemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "cfg or igemm or dgrad_s2" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log; grep -E "FAILED|Error" $O/test.log | head -10
[ $rc -eq 0 ] || exit $rc
DET_IGEMM_CFG=21 timeout -k 10 400 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_igemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "igemm or dgrad_s2 or rs_autograd" > $O/test21.log 2>&1; rc=$?
tail -3 $O/test21.log; grep -E "FAILED|Error" $O/test21.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv_default.jsonl 2> $O/conv.err || { tail $O/conv.err; exit 1; }
DET_IGEMM_CFG=21 timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv_cfg21.jsonl 2> $O/conv21.err || { tail $O/conv21.err; exit 1; }
python - <<'PY'
import json
a=[json.loads(l) for l in open("gpurun_out/r6s28/conv_default.jsonl")]
b=[json.loads(l) for l in open("gpurun_out/r6s28/conv_cfg21.jsonl")]
for x,y in zip(a,b):
    if "c" in x:
        print(x["c"], x["stride"], x["hin"], "fwd", x["fwd_native"], "->", y["fwd_native"], "dgrad", x["dgrad_native"], "->", y["dgrad_native"])
    else:
        print("totals", x, y)
PY
