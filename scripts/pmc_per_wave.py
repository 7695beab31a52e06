"""Per-kernel counter totals per wave from a rocprofv3 --pmc counter-collection CSV: every counter
in the run, summed over a kernel's dispatches and divided by its SQ_WAVES (instructions per wave,
cycles per wave, ...).

    python scripts/pmc_per_wave.py pmc_counter_collection.csv [--top 25] [--out FILE]
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"Kind<[^>]*>(, (Kind<[^>]*>|NoKind))?", name)
    if m:
        return name.split("<")[0].replace("void ", "") + "<" + m.group(0) + ">"
    return re.sub(r"\(.*", "", name).replace("void ", "")[:90]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(args.csv, newline="") as f:
        for r in csv.DictReader(f):
            k = short(r.get("Kernel_Name", "?"))
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id"))
    counters = sorted({c for d in tot.values() for c in d if c != "SQ_WAVES"})
    rows = sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("SQ_BUSY_CYCLES", 0)))
    lines = ["kernel | dispatches | waves/dispatch | " + " | ".join(f"{c}/wave" for c in counters)]
    for k, d in rows[:args.top]:
        w = d.get("SQ_WAVES", 0) or 1
        n = len(disp[k]) or 1
        lines.append(f"{k} | {n} | {w / n:.0f} | " + " | ".join(f"{d.get(c, 0) / w:.0f}" for c in counters))
    text = "\n".join(lines)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
