#!/bin/bash
# Round-6 session 30: igemm8 512x128 (cfg 22): numerics on the cfg test shapes, then the ResNet-50
# 3x3 pass timings with cfg 22 forced (where N % 128 == 0) vs the defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s30; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "cfg" > $O/test.log 2>&1; rc=$?
tail -2 $O/test.log; grep -E "FAILED|Error" $O/test.log | head -10
[ $rc -eq 0 ] || exit $rc
DET_IGEMM_CFG=22 timeout -k 10 400 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_igemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "igemm or dgrad_s2 or rs_autograd" > $O/test22.log 2>&1; rc=$?
tail -2 $O/test22.log; grep -E "FAILED|Error" $O/test22.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv_default.jsonl 2> $O/conv.err || { tail $O/conv.err; exit 1; }
DET_IGEMM_CFG=22 timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv_cfg22.jsonl 2> $O/conv22.err || { tail $O/conv22.err; exit 1; }
python - <<'PY'
import json
a=[json.loads(l) for l in open("gpurun_out/r6s30/conv_default.jsonl")]
b=[json.loads(l) for l in open("gpurun_out/r6s30/conv_cfg22.jsonl")]
for x,y in zip(a,b):
    if "c" in x:
        print(x["c"], x["stride"], x["hin"], "fwd", x["fwd_native"], "->", y["fwd_native"], "dgrad", x["dgrad_native"], "->", y["dgrad_native"], x.get("fwd_igemm3"), y.get("fwd_igemm3"), x.get("dgrad_igemm3"), y.get("dgrad_igemm3"))
    else:
        print("totals", x, y)
PY
