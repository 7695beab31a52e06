#!/bin/bash
# Round-6 session 31: fused gemm8 + GELU epilogue for BERT's FFN-in: tests, then BERT bench A/B
# (DET_GEMM8_FFN 1 / 0) under hipGraph and eager, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s31; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm8_gpu.py tests/test_transformer_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1; rc=$?
tail -2 $O/test.log; grep -E "FAILED|Error" $O/test.log | head -10
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    DET_GEMM8_FFN=$v timeout -k 10 300 python -u scripts/bench_bert.py --steps 100 --warmup 10 --hip-graph > $O/bert_g_$v.$i.json 2> $O/bert.err || { tail $O/bert.err; exit 1; }
    echo "graph gemm8_ffn=$v: $(tail -1 $O/bert_g_$v.$i.json | cut -c1-120)"
    DET_GEMM8_FFN=$v timeout -k 10 300 python -u scripts/bench_bert.py --steps 100 --warmup 10 > $O/bert_e_$v.$i.json 2> $O/bert.err || { tail $O/bert.err; exit 1; }
    echo "eager gemm8_ffn=$v: $(tail -1 $O/bert_e_$v.$i.json | cut -c1-120)"
  done
done
