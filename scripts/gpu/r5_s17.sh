#!/bin/bash
# Round-5 session 17: ASHA trials/hr at the reference adaptive.yaml shape (16 trials, 32 epochs max,
# validation every epoch), 1 GPU slot, O0 and O2 on the native CIFAR kernels with 20-batch graphs;
# then O0 again with cold-exec containers under rocprofv3 for a kernel-trace GPU-busy figure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s17
mkdir -p $O
export TMPDIR=/tmp
for amp in O0 O2; do
  DET_BENCH_LOGDIR=$O timeout -k 10 900 python -u scripts/bench_asha.py --slots 1 --amp $amp --graph-batches 20 --timeout 840 \
    > $O/asha_$amp.json 2> $O/asha_$amp.err || { echo "asha $amp rc=$?"; tail -20 $O/asha_$amp.err; exit 1; }
  echo "asha $amp: $(grep '^{' $O/asha_$amp.json | tail -1 | cut -c1-600)"
done
DET_BENCH_LOGDIR=/tmp timeout -k 10 900 rocprofv3 --kernel-trace -d /tmp/aprof -o asha -- python3 -u scripts/bench_asha.py \
  --slots 1 --amp O0 --graph-batches 20 --timeout 840 --no-zygote > $O/asha_prof.json 2> $O/asha_prof.err \
  || { echo "asha prof rc=$?"; tail -20 $O/asha_prof.err; exit 1; }
echo "asha prof: $(grep '^{' $O/asha_prof.json | tail -1 | cut -c1-400)"
python3 scripts/prof_busy.py /tmp/aprof --out $O/asha_o0_rocprof_busy.json
