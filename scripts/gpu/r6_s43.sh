#!/bin/bash
# Round-6 session 43: per-kernel hardware counters of the ResNet-50 step with the igemm8 convs
# (eager steps: counter collection serialises dispatches), summarised by scripts/pmc_summarize.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s43; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 500 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/pmc -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 2 --no-hip-graph > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
f=$(find $O/pmc -name "pmc_counter_collection.csv" | head -1)
python3 scripts/pmc_summarize.py $f --top 40 --out $O/pmc_summary.csv > $O/pmc_summary.txt 2>&1
head -45 $O/pmc_summary.txt
