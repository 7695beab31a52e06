#!/bin/bash
# Round-6 session 36: wgrad8 (eight-phase ring weight gradient, cfg 14): exactness on the wgrad test
# shapes, then the 3x3 pass timings with DET_WGRAD_CFG=14 forced where it fits vs the defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s36; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > $O/test.log 2>&1; rc=$?
tail -2 $O/test.log; grep -E "FAILED|Error|assert" $O/test.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv_default.jsonl 2> $O/conv.err || { tail $O/conv.err; exit 1; }
DET_WGRAD_CFG=14 timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv_wg14.jsonl 2> $O/conv14.err || { tail $O/conv14.err; exit 1; }
python - <<'PY'
import json
a=[json.loads(l) for l in open("gpurun_out/r6s36/conv_default.jsonl")]
b=[json.loads(l) for l in open("gpurun_out/r6s36/conv_wg14.jsonl")]
for x,y in zip(a,b):
    if "c" in x:
        print(x["c"], x["stride"], x["hin"], "wgrad", x["wgrad_native"], "->", y["wgrad_native"])
    else:
        print("totals", x["totals_ms_per_step"].get("wgrad_native"), y["totals_ms_per_step"].get("wgrad_native"))
PY
