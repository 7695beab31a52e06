"""Print the top entries of a cProfile dump: python scripts/cprof_summary.py file.cprof [N]"""
import pstats
import sys

n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
st = pstats.Stats(sys.argv[1])
st.sort_stats("tottime").print_stats(n)
st.sort_stats("cumulative").print_stats(n)
