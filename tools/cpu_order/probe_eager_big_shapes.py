"""Spot checks of the eager matmul selection at long-prompt prefill shapes (up to 2 001 queries x
2 001 keys, 8 heads): appended to eager_table_2b2b.jsonl. All E/O-32 with no K split."""
import sys, json
import os; _H = os.path.dirname(os.path.abspath(__file__)); sys.path.insert(0, _H); sys.path.insert(0, os.path.dirname(os.path.dirname(_H)))
from probe_eager_table import probe
for (op, M, K, N) in [("pv", 300, 300, 256), ("pv", 602, 602, 256), ("qk", 602, 256, 602), ("pv", 602, 60, 256),
                      ("pv", 1200, 1200, 256), ("qk", 2001, 256, 2001), ("pv", 2001, 2001, 256)]:
    r = probe(M, K, N, H=8)
    print(json.dumps({"op": op, "M": M, "K": K, "N": N, "models": r}), flush=True)
