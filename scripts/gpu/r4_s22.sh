#!/bin/bash
# Round-4 session 22: session 21 showed every hipGraph-chunk run going NaN in the chunk holding the
# first epoch boundary (batch 1563, a 16-record tail batch).  Short epochs (100 full batches + a
# 16-record tail), dropout 0: per-batch losses of eager vs per-batch graphs vs 20-batch chunks.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s22
mkdir -p $O
export TMPDIR=/tmp
for cfg in "O0_eager:--amp O0" "O0_g1:--amp O0 --hip-graph --graph-batches 1" "O0_g20:--amp O0 --hip-graph --graph-batches 20" "O2_eager:--amp O2" "O2_g20:--amp O2 --hip-graph --graph-batches 20"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 180 python -u scripts/bench_cifar_trial.py --batch 32 --batches 320 --chunk 160 --train-records 3216 \
    --lr 1e-4 --seed 1 --no-dropout --batch-losses $args > $O/$name.json 2> $O/$name.err || { tail -30 $O/$name.err; exit 1; }
done
python3 - <<'PY'
import json, math
O = "gpurun_out/r4s22"
for amp, runs in (("O0", ("g1", "g20")), ("O2", ("g20",))):
    e = json.load(open(f"{O}/{amp}_eager.json"))["batch_losses"]
    for m in runs:
        d = json.load(open(f"{O}/{amp}_{m}.json"))
        b = d["batch_losses"]
        bad = next((i for i, (x, y) in enumerate(zip(e, b)) if not math.isfinite(y) or abs(x - y) > 0.05), None)
        print(amp, m, d["hip_graph"], "first batch off by >0.05 or non-finite:", bad)
        if bad is not None:
            print("  eager", [round(x, 4) for x in e[max(0, bad - 3):bad + 4]])
            print("  " + m, [round(x, 4) if math.isfinite(x) else x for x in b[max(0, bad - 3):bad + 4]])
PY
