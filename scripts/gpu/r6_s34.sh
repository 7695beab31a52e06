#!/bin/bash
# Round-6 session 34: igemm8 for the measured 1x1 shapes: conv tests, bench A/B (DET_IGEMM8 1 / 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s34; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_igemm_gpu.py tests/test_bn_bwd_fusion_gpu.py tests/test_conv_gpu.py tests/test_conv2d_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1; rc=$?
tail -2 $O/test.log; grep -E "FAILED|Error" $O/test.log | head -10
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    DET_IGEMM8=$v timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 > $O/bench_i8_$v.$i.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
    echo "igemm8=$v: $(tail -1 $O/bench_i8_$v.$i.json | cut -c1-140)"
  done
done
