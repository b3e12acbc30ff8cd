"""Summarise an HZ_STREAM_TRACE file (hz_fb_stream.hip trace_flush): per launch kind, the span from
the first workgroup's start to the last workgroup's end, and the gaps between consecutive launches
(the last workgroup's end of one to the first workgroup's start of the next), in microseconds."""
import collections
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
rec = 8 + 1024 * 8
n = len(raw) // rec
kinds, spans, starts, ends = [], [], [], []
for i in range(n):
    k, wg = np.frombuffer(raw, dtype=np.int32, count=2, offset=i * rec)
    st = np.frombuffer(raw, dtype=np.uint64, count=1024, offset=i * rec + 8)
    s0, e0 = st[:wg], st[512:512 + wg]
    kinds.append(int(k))
    starts.append(int(s0.min()))
    ends.append(int(e0.max()))
names = {0: "block", 1: "block+transient", 2: "setter"}
print(f"{n} launches")
span = collections.defaultdict(list)
for k, s, e in zip(kinds, starts, ends):
    span[names[k]].append((e - s) / 100.0)
for k, v in span.items():
    print(f"  {k:16s} n={len(v):5d} span mean {np.mean(v):6.2f} median {np.median(v):6.2f} us")
gaps = collections.defaultdict(list)
for i in range(1, n):
    g = (starts[i] - ends[i - 1]) / 100.0
    if g < 1000:   # (between separate passes: host time)
        gaps[(names[kinds[i - 1]], names[kinds[i]])].append(g)
for k, v in gaps.items():
    print(f"  gap {k[0]:16s} -> {k[1]:16s} n={len(v):5d} mean {np.mean(v):6.2f} median {np.median(v):6.2f} us")
# the churn pass: from the first setter to the last launch
f = kinds.index(2)
tot = (ends[-1] - starts[f]) / 100.0
nb = sum(1 for k in kinds[f:] if k != 2)
print(f"  from the first setter: {tot:.1f} us over {nb} blocks = {tot / max(1, nb):.2f} us per block")
