#!/bin/bash
# Round-5 session 38: attention workgroups of 2 waves (64 query rows; 864 workgroups at the BERT
# shape instead of 432 on 256 CUs) vs 4 waves: attention tests, attention microbench, BERT graph.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s38
mkdir -p $O
export TMPDIR=/tmp
L2=$PWD/determined_1_amd/ops/libdetkernels_attn2.so
DET_KERNELS_LIB=$L2 timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -q --timeout 200 --timeout-method thread > $O/tests2.log 2>&1 || { tail -30 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
for lib in default attn2 default attn2; do
  env_lib=""; [ "$lib" = "attn2" ] && env_lib="DET_KERNELS_LIB=$L2"
  env $env_lib timeout -k 10 200 python -u scripts/bench_attn.py > $O/attn_$lib.json 2> $O/attn.err || { tail -20 $O/attn.err; exit 1; }
  echo "attn $lib: $(cut -c1-300 $O/attn_$lib.json)"
  env $env_lib timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 --hip-graph > $O/bert.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
  echo "bert graph $lib: $(grep -o '"value": [0-9.]*' $O/bert.json)"
done
