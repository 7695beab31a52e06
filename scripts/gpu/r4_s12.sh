#!/bin/bash
# Round-4 session 12: BN statistics epilogues moved after the C stores (every GEMM with STATS),
# 32-bit index math in the stride-2 residual gather and the 1x1 stride-2 row gather; the BERT
# resume / dropout-stream / hipGraph-refusal tests; bench x2 and the roofline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_conv_gpu.py tests/test_igemm_gpu.py tests/test_conv3x3_gpu.py tests/test_bn_bwd_fusion_gpu.py tests/test_pool_gpu.py tests/test_norm_gpu.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_bert_trial_resume.py > $O/pytest_bert_resume.log 2>&1 || { tail -40 $O/pytest_bert_resume.log; exit 1; }
tail -1 $O/pytest_bert_resume.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_$i.json 2> $O/bench_$i.err || { tail -30 $O/bench_$i.err; exit 1; }
  echo "bench $i $(python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 300 python -u scripts/step_roofline.py --iters 3 --out $O/step_roofline.csv > $O/step_roofline.txt 2>&1 || { tail -30 $O/step_roofline.txt; exit 1; }
sed -n '/per family/,$p' $O/step_roofline.txt | head -34
