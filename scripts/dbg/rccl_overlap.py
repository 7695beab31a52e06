"""From a rocprofv3 rocpd DB of a data-parallel step: the RCCL kernels (names containing nccl),
their streams, and how much of their time overlaps compute kernels on other streams."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
ks = c.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
comm = [k for k in ks if "nccl" in k[0].lower() or "rccl" in k[0].lower()]
comp = [k for k in ks if k not in comm]
print(f"kernels {len(ks)}  rccl kernels {len(comm)}  rccl busy {sum(k[2] - k[1] for k in comm) / 1e6:.2f} ms")
names = {}
for k in comm:
    names.setdefault(k[0][:90], [0, 0.0])
    names[k[0][:90]][0] += 1
    names[k[0][:90]][1] += (k[2] - k[1]) / 1e6
for n, (cnt, ms) in sorted(names.items(), key=lambda x: -x[1][1])[:10]:
    print(f"  {ms:8.2f} ms {cnt:5d}  {n}")
print("rccl streams", sorted({k[3] for k in comm}), "compute streams", sorted({k[3] for k in comp})[:8])
# overlap: merge compute intervals, intersect with each comm kernel
iv = []
for k in comp:
    if iv and k[1] <= iv[-1][1]:
        iv[-1][1] = max(iv[-1][1], k[2])
    else:
        iv.append([k[1], k[2]])
import bisect
starts = [a for a, _ in iv]
ov = 0
tot = 0
for k in comm:
    s, e = k[1], k[2]
    tot += e - s
    i = max(0, bisect.bisect_right(starts, s) - 1)
    while i < len(iv) and iv[i][0] < e:
        a, b = iv[i]
        ov += max(0, min(b, e) - max(a, s))
        i += 1
print(f"rccl time overlapped with compute: {ov / 1e6:.2f} of {tot / 1e6:.2f} ms ({100 * ov / max(1, tot):.1f}%)")
