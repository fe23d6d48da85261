#!/usr/bin/env python3
"""Error table of a GPU test run: every measured error beside its bound.

The GPU tests append one JSON line per comparison to $ACE_ERROR_LOG
(tests/conftest.py record_error): the referee's gradient / stats / mu
errors, the prediction variances and ATE/ATT/ATU intervals against the
oracle, the multi-process mu, and for every `close()` call the fraction of
its bound the worst element used.  This groups them by test function and
check, and prints the largest measured value, the bound and their ratio
(headroom = bound / max measured; a bound more than 5x the largest
measured error is marked).

Usage: python tools/error_table.py ERROR_LOG.jsonl > profiles/rNN_error_table.txt
"""
import collections
import json
import sys


def main():
    rows = collections.defaultdict(list)
    for line in open(sys.argv[1]):
        d = json.loads(line)
        fn = d["test"].split("[")[0]
        rows[(fn, d["check"], d["bound"])].append((d["measured"], d["test"]))
    print(f"{'test function':58s} {'check':62s} {'n':>4s} {'max measured':>12s} {'bound':>9s} {'headroom':>9s}")
    loose = 0
    for (fn, check, bound), v in sorted(rows.items()):
        m, worst = max(v)
        head = bound / m if m > 0 else float("inf")
        flag = "  >5x" if head > 5 else ""
        loose += head > 5
        print(f"{fn:58s} {check:62s} {len(v):4d} {m:12.3e} {bound:9.2e} {head:9.1f}{flag}")
    print(f"\n{len(rows)} checks; {loose} with a bound more than 5x the largest measured value "
          "(the north-star 1e-6 comparisons against the fp64 oracle stay at the spec)")


if __name__ == "__main__":
    main()
