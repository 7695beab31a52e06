#!/bin/bash
# Round-3 session 40: layer1 projection-shortcut gradient linked into the stem max-pool backward
# (summed in the gather kernel; no autograd add pass): kernel/link tests, bench A/B, GPU tier, smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s40
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_pool_gpu.py tests/test_conv_gpu.py tests/test_norm_gpu.py > $O/pytest_pool.log 2>&1 || { tail -40 $O/pytest_pool.log; exit 1; }
tail -1 $O/pytest_pool.log
for v in 1 0 1 0; do
  DET_MAXPOOL_LINK=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_link$v.json 2> $O/bench_link$v.err || { tail -30 $O/bench_link$v.err; exit 1; }
  echo "link=$v $(cut -c1-140 $O/bench_link$v.json)"
done
