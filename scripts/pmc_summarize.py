"""Per-kernel summary of a rocprofv3 --pmc counter-collection CSV (one row per dispatch x counter).

    python scripts/pmc_summarize.py run_counter_collection.csv [--top 30] [--out summary.csv]

Sums every counter per kernel name over its dispatches and prints, per kernel, the SQ cycle split
(SQ_WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY, all in quad-cycles), the LDS
issue-stall and bank-conflict shares, and the MFMA busy cycles per GRBM_GUI_ACTIVE cycle per CU
(GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES over all SIMDs, so the
matrix cores of a CU are saturated at 4 per CU-cycle -- the value is reported as a fraction of 4).
Kernels are ranked by GRBM_GUI_ACTIVE (time-weighted), counter names absent from the run are
skipped."""
import argparse
import csv
import collections
import sys

NCU = 256


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(args.csv, newline="") as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name") or row.get("KernelName") or "?"
            cn = row.get("Counter_Name") or row.get("CounterName")
            cv = row.get("Counter_Value") or row.get("CounterValue")
            if cn is None or cv is None:
                continue
            try:
                tot[name][cn] += float(cv)
            except ValueError:
                continue
            disp[name].add(row.get("Dispatch_Id") or row.get("DispatchId") or row.get("Correlation_Id"))
    if not tot:
        print("no counter rows", file=sys.stderr)
        sys.exit(1)

    def key(k):
        c = tot[k]
        return c.get("GRBM_GUI_ACTIVE", c.get("SQ_WAVE_CYCLES", 0.0))

    rows = []
    for k in sorted(tot, key=key, reverse=True):
        c = tot[k]
        wave = c.get("SQ_WAVE_CYCLES", 0.0)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        r = {"kernel": k[:110], "dispatches": len(disp[k])}
        if wave > 0:
            for cn, lab in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst"),
                            ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_WAIT_INST_LDS", "wait_lds")):
                if cn in c:
                    r[lab] = round(c[cn] / wave, 3)
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE", 0) > 0:
            r["lds_conflict"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 3)
        elif "SQ_LDS_BANK_CONFLICT" in c and wave > 0:
            r["lds_conflict_per_wave_cyc"] = round(c["SQ_LDS_BANK_CONFLICT"] / wave, 4)
        if gui > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            r["mfma_util"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / 8 * NCU) / 4, 3)
        if gui > 0:
            r["gui_active_M"] = round(gui / 1e6, 2)
        # memory-side traffic (KB summed over dispatches; gfx950 FETCH_SIZE counts 64 B per 128-B
        # request of a wide streaming read, so it is doubled -- MI355X_MICROARCH.md)
        if "FETCH_SIZE" in c:
            r["fetch_MB"] = round(2 * c["FETCH_SIZE"] / 1024.0, 1)
        if "WRITE_SIZE" in c:
            r["write_MB"] = round(c["WRITE_SIZE"] / 1024.0, 1)
        hit, miss = c.get("TCC_HIT_sum", c.get("TCC_HIT")), c.get("TCC_MISS_sum", c.get("TCC_MISS"))
        if hit is not None and miss is not None and hit + miss > 0:
            r["l2_hit"] = round(hit / (hit + miss), 3)
        if disp[k]:
            r["dispatches"] = len(disp[k])
        rows.append(r)
    cols = ["kernel", "dispatches", "gui_active_M", "mfma_util", "wait_any", "wait_inst", "active", "wait_lds",
            "lds_conflict", "lds_conflict_per_wave_cyc", "fetch_MB", "write_MB", "l2_hit"]
    cols = [c for c in cols if any(c in r for r in rows)]
    for r in rows[:args.top]:
        print("  ".join(f"{c}={r[c]}" for c in cols if c in r))
    if args.out:
        with open(args.out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=cols)
            w.writeheader()
            for r in rows:
                w.writerow({c: r.get(c, "") for c in cols})


if __name__ == "__main__":
    main()
