#!/bin/bash
# Round-4 session 19: per-kernel memory-side traffic of the ResNet-50 step (two counter passes:
# FETCH_SIZE; WRITE_SIZE + L2 hit/miss), to set against the compulsory bytes of the roofline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s19
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pa -o run -- python3 -u bench.py --steps 2 --warmup 2 > $O/pa.json 2> $O/pa.err || { tail -20 $O/pa.err; exit 1; }
f=$(find $O/pa -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summarize.py "$f" --top 40 --out $O/pmc_fetch.csv > $O/pmc_fetch.txt 2>&1 || { tail -5 $O/pmc_fetch.txt; exit 1; }
head -20 $O/pmc_fetch.txt
rm -rf $O/pa
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/pb -o run -- python3 -u bench.py --steps 2 --warmup 2 > $O/pb.json 2> $O/pb.err || { tail -20 $O/pb.err; exit 1; }
f=$(find $O/pb -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summarize.py "$f" --top 40 --out $O/pmc_write.csv > $O/pmc_write.txt 2>&1 || { tail -5 $O/pmc_write.txt; exit 1; }
head -20 $O/pmc_write.txt
rm -rf $O/pb
