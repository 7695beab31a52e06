"""Summarise a rocprofv3 rocpd SQLite output: kernel count, busy time, top kernels."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, count(*), sum(end-start) from kernels group by name order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"kernels {sum(r[1] for r in rows)} busy_ms {tot / 1e6:.2f}")
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{r[2] / 1e6:9.2f} ms {r[1]:7d} {r[2] / r[1] / 1e3:8.2f} us  {r[0][:110]}")
