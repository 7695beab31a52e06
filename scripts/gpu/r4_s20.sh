#!/bin/bash
# Round-4 session 20: CIFAR trial with dropout 0 -- per-batch losses of eager vs per-batch hipGraph vs
# 20-batch hipGraph chunks at O0 and O2 over 200 batches (session 18: O2 + graph chunks went NaN
# where O2 eager learned), then the session-19 memory-traffic passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s20
mkdir -p $O
export TMPDIR=/tmp
for amp in O0 O2; do
  for cfg in "eager:" "g1:--hip-graph --graph-batches 1" "g20:--hip-graph --graph-batches 20"; do
    name=${amp}_${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 180 python -u scripts/bench_cifar_trial.py --batch 32 --batches 200 --chunk 100 --amp $amp \
      --no-dropout --batch-losses $args > $O/$name.json 2> $O/$name.err || { tail -30 $O/$name.err; exit 1; }
  done
done
python3 - <<'PY'
import json
O = "gpurun_out/r4s20"
for amp in ("O0", "O2"):
    d = {m: json.load(open(f"{O}/{amp}_{m}.json")) for m in ("eager", "g1", "g20")}
    e = d["eager"]["batch_losses"]
    for m in ("g1", "g20"):
        b = d[m]["batch_losses"]
        diff = [abs(x - y) for x, y in zip(e, b)]
        first = next((i for i, x in enumerate(diff) if x > 1e-3), None)
        print(amp, m, "graph", d[m]["hip_graph"], "first batch |dloss|>1e-3:", first,
              "eager[-5:]", [round(x, 4) for x in e[-5:]], m + "[-5:]", [round(x, 4) for x in b[-5:]])
PY
bash scripts/gpu/r4_s19.sh
