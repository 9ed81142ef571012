"""Locate the value-arena bytes where one large-block pass-3 form differs from
another (ablation build): for the first differing blocks, the row, the byte's
place in its row and 16-byte chunk, and the tile owning its source.

usage: python tools/tile_diff.py [armA] [armB]   (arms as in tools/ablate_tile.py)
env:   ABL_NBLK (4096), ABL_KIND (1), ABL_BS (65536), ABL_TH (57344)
"""
import os as _os
_os.environ.setdefault("OKV_ABLATE", "1")

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import objectkv_amd as okv  # noqa: E402

arms = sys.argv[1:3] if len(sys.argv) >= 3 else ["7", "8:16xd7"]
nblk = int(os.environ.get("ABL_NBLK", "4096"))
w = okv.synth_segment(int(os.environ.get("ABL_KIND", "1")), 3, nblocks=nblk,
                      threshold=int(os.environ.get("ABL_TH", "57344")),
                      block_size=int(os.environ.get("ABL_BS", "65536")))
seg, d = w.data(), w.descs()[:nblk]
outs = []
for a in arms:
    vs, _, tile = a.partition(":")
    os.environ["OKV_VALUE_SWEEP"] = vs
    os.environ["OKV_TILE"] = tile or "16x"
    dec = okv.Decoder(0)
    outs.append(dec.decode(seg, d))
    dec.close()
A, B = outs
va, vb = A.val_arena, B.val_arena
print("rows", A.row_start[-1], B.row_start[-1], "vbytes", va.size, vb.size)
diff = np.nonzero(va != vb)[0]
print("differing value bytes:", diff.size)
if diff.size:
    vbase = A.val_base.astype(np.int64)
    blocks = np.unique(np.searchsorted(vbase, diff, side="right") - 1)
    print("blocks with differences:", blocks.size, "first:", blocks[:10])
    import re
    tile = int(re.match(r"\d+", arms[1].partition(":")[2] or "16").group()) * 1024
    for b in blocks[:4]:
        lo = int(vbase[b])
        bd = diff[(diff >= lo) & (diff < (vbase[b + 1] if b + 1 < nblk else va.size))]
        r0, r1 = int(A.row_start[b]), int(A.row_start[b + 1])
        voff = A.val_off[r0:r1].astype(np.int64) - lo
        vlen = A.val_len[r0:r1].astype(np.int64)
        koff = A.key_off[r0:r1].astype(np.int64)
        klen = A.key_len[r0:r1].astype(np.int64)
        # block positions of each row's value (record walk)
        pos, vsrc = 0, []
        for r in range(r1 - r0):
            vsrc.append(pos + 6 + klen[r])
            pos += 6 + klen[r] + vlen[r]
        print(f"block {b}: rows {r1 - r0}, {bd.size} bytes differ, value region {voff[-1] + vlen[-1]}")
        runs = np.split(bd, np.nonzero(np.diff(bd) != 1)[0] + 1)
        for run in runs[:6]:
            x = int(run[0]) - lo
            r = int(np.searchsorted(voff, x, side="right") - 1)
            src = vsrc[r] + x - voff[r]
            print(f"   dest [{x}, {x + run.size}) chunk {x >> 4}+{x & 15}: row {r} "
                  f"[{voff[r]}, {voff[r] + vlen[r]}) src {src} (tile {src // tile} +{src % tile}) "
                  f"A={va[run[0]:run[0] + 4]} B={vb[run[0]:run[0] + 4]}")
