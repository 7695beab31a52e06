#!/bin/bash
# Round-5 session 3: (a) does per-replay synchronisation hide the round-4 O2 graph NaN?  Round-4
# model (element dropout after pool 1, RMSprop alpha 0.99) with checks every replay vs every 200
# replays (asynchronous), torch / fixed-bank / torch.rand masks; the reference model (Dropout2d,
# alpha 0.9) asynchronous.  (b) the native CIFAR CNN kernels against the fp32 torch reference.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s3
mkdir -p $O
export TMPDIR=/tmp
for cfg in "r4_torch_c1:--variant torch --r4-model" "r4_torch_c200:--variant torch --r4-model --check-every 200" \
           "r4_bank_c200:--variant bankmask --r4-model --check-every 200" "r4_rand_c200:--variant randmask --r4-model --check-every 200" \
           "ref_torch_c200:--variant torch --check-every 200" "r4_torch_c200_s2:--variant torch --r4-model --check-every 200 --seed 2"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 240 python -u scripts/dbg/graph_nan_probe.py $a --batches 2400 --out $O > $O/$name.json 2> $O/$name.err \
    || { echo "$name failed rc=$?"; tail -30 $O/$name.err; exit 1; }
  echo "== $name"; cut -c1-600 $O/$name.json
done
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -x -v --timeout 120 --timeout-method thread > $O/cnn_tests.log 2>&1
rc=$?; tail -40 $O/cnn_tests.log; exit $rc
