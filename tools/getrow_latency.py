"""GetRow cost through the product reader (okv_reader.cpp): every call is one
host-mode GPU decode of the one block the btree floor picks (H2D of the
block, plan, decode, D2H of its rows) -- what a Go GetRow pays through the cgo
shim.  Also the bare host-mode okv_decode_plan +
okv_decode_blocks of one block, and a RowIter scan for comparison.

usage: python tools/getrow_latency.py [calls]   -> one JSON line"""
import json
import os
import random
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import objectkv_amd as okv  # noqa: E402
from objectkv_amd import reader as R  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dec = okv.Decoder(0)
res = {}
for name, kind, nblk, th, bs in (("4KiB_blocks", okv.sst.SYNTH_FIXED, 2048, 3584, 4096),
                                 ("64KiB_blocks", okv.sst.SYNTH_ZIPF, 2048, 57344, 65536)):
    w = okv.synth_segment(kind, 3, nblocks=nblk, threshold=th, block_size=bs)
    data = w.data().tobytes()
    d = w.descs()
    pr = R.SegmentReader(data, len(data), dec)
    n = pr.NumBlocks()
    keys = []
    rng = random.Random(1)
    for i in rng.sample(range(n - 1), 16):
        rows = pr.ReadBlock(i)
        keys.append(rows[len(rows) // 2].Key)
    for k in keys[:4]:  # warm
        pr.GetRow(k)
    t = []
    for c in range(calls):
        k = keys[c % len(keys)]
        t0 = time.perf_counter()
        got = pr.GetRow(k)
        t.append((time.perf_counter() - t0) * 1e6)
        assert got.Key == k
    seg = np.frombuffer(data, np.uint8)
    one = []
    for c in range(calls):
        b = rng.randrange(n - 1)
        t0 = time.perf_counter()
        dec.decode(seg[int(d[b, 0]):int(d[b, 0] + d[b, 1])], np.array([[0, d[b, 1], d[b, 2], 0]],
                                                                       np.uint64))
        one.append((time.perf_counter() - t0) * 1e6)
    it = pr.RowIter(0)
    t0 = time.perf_counter()
    m = 0
    while True:
        try:
            it.Next()
            m += 1
        except R.GoError:
            break
    scan = time.perf_counter() - t0
    res[name] = {"getrow_us_median": round(statistics.median(t), 1),
                 "getrow_us_p90": round(sorted(t)[int(0.9 * len(t))], 1),
                 "decode_one_block_host_us_median": round(statistics.median(one), 1),
                 "block_bytes": int(d[0, 1]), "rowiter_rows_per_s": round(m / scan),
                 "io_stats": pr.io_stats()}
print(json.dumps(res), flush=True)
